// mh_bgzf.h — host side of the BAM writer: BGZF framing on a deflate thread pool and the BAI index (SAM/BAM
// specification §4.1 / §5.2; the reference produces these through htslib via pysam.sort / pysam.index,
// god_aligner.py:117-131).  The BAI is a valid spec index of our own file, not byte-identical to htslib's output
// (htslib's chunk merging and linear-index fill are not pinned here: no htslib in the image).  Plain C++ (no HIP); compiled with g++ and linked against zlib.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace mh {

constexpr int64_t BGZF_BLOCK = 0xff00;   // uncompressed bytes per block (htslib BGZF_BLOCK_SIZE)

struct BaiRec {   // one record, coordinate-sorted
  int32_t tid, beg, end;
  uint32_t bin;
};

// BAM header bytes: magic, l_text, text, n_ref, (l_name, name\0, l_ref) per reference.
std::string bam_header_bytes(const std::string &text, const std::vector<std::string> &names,
                             const std::vector<int64_t> &lens);

// Writes a BGZF file: `header` (own block(s), as htslib flushes after the header), then `data` cut into
// BGZF_BLOCK-byte blocks, then the EOF marker.  rec_block_coff[b] = file offset of data block b
// (b = 0..nblocks; the last entry is the offset of the EOF block).  Returns false and sets err on failure.
bool bgzf_write(const char *path, const std::string &header, const uint8_t *data, int64_t n, int level, int threads,
                std::vector<int64_t> &rec_block_coff, std::string &err);

// The same file from data blocks deflated elsewhere (the device, mh_bam_write_gpu): `header` deflated here at `level`
// in its own block(s), then n_z bytes of ready BGZF blocks fetched in pieces, then the EOF
// marker.  boff[b] = offset of data block b inside those bytes (b = 0..nblocks); rec_block_coff as bgzf_write's.
// fetch(offset, len) returns host bytes [offset, offset + len) (len <= 64 MiB), valid until the next call, or null.
bool bgzf_write_blocks(const char *path, const std::string &header, int level, int64_t n_z,
                       const std::vector<int64_t> &boff,
                       const std::function<const uint8_t *(int64_t, int64_t)> &fetch,
                       std::vector<int64_t> &rec_block_coff, std::string &err);

// The same file with the data blocks handed over as they are ready: next(&buf, &len) gives the next piece of BGZF
// bytes (false: no more).  *data_pos = the data's file offset (after the header block(s)), *end_pos = the EOF
// marker's.
// eof false: no EOF marker (a part of a file other writers complete, mh_bam_write_part).
bool bgzf_write_stream(const char *path, const std::string &header, int level,
                       const std::function<bool(const uint8_t **, int64_t *)> &next, int64_t *data_pos,
                       int64_t *end_pos, std::string &err, bool eof = true);

// BAI for n sorted records whose data offsets are soff[0..n] (soff[n] = end), given the block map from bgzf_write.
bool bai_write(const char *path, int32_t n_refs, int64_t n, const BaiRec *recs, const int64_t *soff,
               const std::vector<int64_t> &rec_block_coff, std::string &err);

// The BAI in two halves, so the per-record half runs before the blocks' file offsets are known (beside the device
// deflate): bai_plan, on `threads` threads, finds per reference the chunks (runs of consecutive records in one bin)
// and the linear index as record indices; bai_emit maps them to virtual offsets and writes the file.
// Every position below indexes bai_emit's `offs` array: the records' data offsets (bai_plan: offs = soff, positions
// = record indices) or a compact array of just the offsets the index needs (the device plan, mh_bam.hip).
struct BaiRun {
  uint32_t bin;
  int64_t kb, ke;   // a chunk: from the offset at kb to the offset at ke (records [kb, ke) for bai_plan)
};
struct BaiRef {
  int64_t n = 0;               // records on the reference
  int64_t vi = 0, vj = 0;      // positions of its first record's offset and of its end
  std::vector<BaiRun> runs;    // by bin, then record order
  std::vector<int64_t> lin;    // per 16 kbp window: the position of its first overlapping record's offset, or -1
};
struct BaiPlan {
  std::vector<BaiRef> refs;
};
bool bai_plan(int32_t n_refs, int64_t n, const BaiRec *recs, int threads, BaiPlan &plan, std::string &err);
bool bai_emit(const char *path, const BaiPlan &plan, const int64_t *offs, const std::vector<int64_t> &rec_block_coff,
              std::string &err);

// virtual offset of data offset u
inline uint64_t voffset(const std::vector<int64_t> &coff, int64_t u) {
  const int64_t b = u / BGZF_BLOCK;
  return (uint64_t)coff[b] << 16 | (uint64_t)(u - b * BGZF_BLOCK);
}

}  // namespace mh
