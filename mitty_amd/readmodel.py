"""Read-model loading: the `.pkl` data contract without unpickling.

The reference resolves a model name in `get_read_model` (reference `mitty/cli.py:255-278`): a built-in name
under `mitty/data/readmodels/` first, otherwise a literal path, then `pickle.load` and a dispatch on
`model['model_class']` (only `'illumina'` exists).  The `.pkl` schema is written by
`mitty/empirical/bam2illumina.py:116-129`: a dict of scalars plus numpy arrays
(`bq_mat` u64[2,max_bp,94], `cum_bq_mat` f64[2,max_bp,94], `tlen` u64[max_tlen], `cum_tlen` f64[max_tlen]).

We never run `pickle.load` on a model file.  `parse_model_pickle` walks the pickle opcode stream as *data*:
it recognises exactly the opcodes those files use and the three numpy globals that describe an ndarray
(`_reconstruct`, `ndarray`, `dtype`), rebuilds the arrays from their raw bytes with `numpy.frombuffer`, and
refuses every other global.  Nothing named in the file is imported or called.

The five built-in models ship as `mitty_amd/data/readmodels/<name>.npz` (converted once from the reference's
`.pkl` files with this parser; loaded with `allow_pickle=False`).
"""
import io
import os
import struct

import numpy as np

BUILTIN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'readmodels')


class UnsafeModelError(ValueError):
  """The pickle names something other than plain data + numpy arrays."""


class _Sym:
  __slots__ = ('module', 'name')

  def __init__(self, module, name):
    self.module, self.name = module, name

  def __repr__(self):
    return '_Sym({}.{})'.format(self.module, self.name)


class _ArrayStub:
  """Result of REDUCE(_reconstruct, (ndarray, (0,), b'b')): an ndarray awaiting its BUILD state."""
  __slots__ = ('value',)

  def __init__(self):
    self.value = None


class _DtypeStub:
  __slots__ = ('base', 'value')

  def __init__(self, base):
    self.base, self.value = base, None


_RECONSTRUCT = {('numpy.core.multiarray', '_reconstruct'), ('numpy._core.multiarray', '_reconstruct')}
_SCALAR = {('numpy.core.multiarray', 'scalar'), ('numpy._core.multiarray', 'scalar')}
_ALLOWED = _RECONSTRUCT | _SCALAR | {('numpy', 'ndarray'), ('numpy', 'dtype')}

_MARK = object()


def _finish(x):
  if isinstance(x, _ArrayStub):
    if x.value is None:
      raise UnsafeModelError('ndarray without state')
    return x.value
  if isinstance(x, _DtypeStub):
    return x.value if x.value is not None else np.dtype(x.base)
  if isinstance(x, dict):
    return {_finish(k): _finish(v) for k, v in x.items()}
  if isinstance(x, list):
    return [_finish(v) for v in x]
  if isinstance(x, tuple):
    return tuple(_finish(v) for v in x)
  if isinstance(x, _Sym):
    raise UnsafeModelError('bare global {!r} in model data'.format(x))
  return x


def _dtype_of(d):
  if isinstance(d, _DtypeStub):
    return d.value if d.value is not None else np.dtype(d.base)
  raise UnsafeModelError('array state without a dtype')


def parse_model_pickle(data):
  """Decode a read-model pickle (protocol 2-4 subset) into Python data without executing anything."""
  f = io.BytesIO(data)
  stack, memo = [], {}

  def pop_mark():
    items = []
    while True:
      v = stack.pop()
      if v is _MARK:
        break
      items.append(v)
    items.reverse()
    return items

  read = f.read
  while True:
    op = read(1)
    if not op:
      raise UnsafeModelError('truncated pickle')
    c = op[0]
    if c == 0x80:      # PROTO
      read(1)
    elif c == 0x95:    # FRAME
      read(8)
    elif c == 0x2e:    # STOP
      break
    elif c == 0x7d:    # EMPTY_DICT
      stack.append({})
    elif c == 0x5d:    # EMPTY_LIST
      stack.append([])
    elif c == 0x29:    # EMPTY_TUPLE
      stack.append(())
    elif c == 0x28:    # MARK
      stack.append(_MARK)
    elif c == 0x71:    # BINPUT
      memo[read(1)[0]] = stack[-1]
    elif c == 0x72:    # LONG_BINPUT
      memo[struct.unpack('<I', read(4))[0]] = stack[-1]
    elif c == 0x94:    # MEMOIZE
      memo[len(memo)] = stack[-1]
    elif c == 0x68:    # BINGET
      stack.append(memo[read(1)[0]])
    elif c == 0x6a:    # LONG_BINGET
      stack.append(memo[struct.unpack('<I', read(4))[0]])
    elif c == 0x58:    # BINUNICODE
      n = struct.unpack('<I', read(4))[0]
      stack.append(read(n).decode('utf-8', 'surrogatepass'))
    elif c == 0x8c:    # SHORT_BINUNICODE
      n = read(1)[0]
      stack.append(read(n).decode('utf-8', 'surrogatepass'))
    elif c == 0x42:    # BINBYTES
      n = struct.unpack('<I', read(4))[0]
      stack.append(read(n))
    elif c == 0x43:    # SHORT_BINBYTES
      n = read(1)[0]
      stack.append(read(n))
    elif c == 0x8e:    # BINBYTES8
      n = struct.unpack('<Q', read(8))[0]
      stack.append(read(n))
    elif c == 0x4a:    # BININT
      stack.append(struct.unpack('<i', read(4))[0])
    elif c == 0x4b:    # BININT1
      stack.append(read(1)[0])
    elif c == 0x4d:    # BININT2
      stack.append(struct.unpack('<H', read(2))[0])
    elif c == 0x8a:    # LONG1
      n = read(1)[0]
      stack.append(int.from_bytes(read(n), 'little', signed=True))
    elif c == 0x47:    # BINFLOAT
      stack.append(struct.unpack('>d', read(8))[0])
    elif c == 0x4e:    # NONE
      stack.append(None)
    elif c == 0x88:    # NEWTRUE
      stack.append(True)
    elif c == 0x89:    # NEWFALSE
      stack.append(False)
    elif c == 0x74:    # TUPLE
      stack.append(tuple(pop_mark()))
    elif c == 0x85:    # TUPLE1
      stack[-1] = (stack[-1],)
    elif c == 0x86:    # TUPLE2
      b = stack.pop(); a = stack.pop(); stack.append((a, b))
    elif c == 0x87:    # TUPLE3
      cc = stack.pop(); b = stack.pop(); a = stack.pop(); stack.append((a, b, cc))
    elif c == 0x73:    # SETITEM
      v = stack.pop(); k = stack.pop(); stack[-1][k] = v
    elif c == 0x75:    # SETITEMS
      items = pop_mark()
      d = stack[-1]
      for i in range(0, len(items), 2):
        d[items[i]] = items[i + 1]
    elif c == 0x61:    # APPEND
      v = stack.pop(); stack[-1].append(v)
    elif c == 0x65:    # APPENDS
      items = pop_mark(); stack[-1].extend(items)
    elif c == 0x63:    # GLOBAL
      module = f.readline()[:-1].decode('ascii')
      name = f.readline()[:-1].decode('ascii')
      if (module, name) not in _ALLOWED:
        raise UnsafeModelError('model pickle references {}.{}: refused'.format(module, name))
      stack.append(_Sym(module, name))
    elif c == 0x93:    # STACK_GLOBAL
      name = stack.pop(); module = stack.pop()
      if (module, name) not in _ALLOWED:
        raise UnsafeModelError('model pickle references {}.{}: refused'.format(module, name))
      stack.append(_Sym(module, name))
    elif c == 0x52:    # REDUCE
      args = stack.pop(); fn = stack.pop()
      if not isinstance(fn, _Sym):
        raise UnsafeModelError('REDUCE on a non-global')
      key = (fn.module, fn.name)
      if key in _RECONSTRUCT:
        if not (isinstance(args, tuple) and len(args) == 3 and isinstance(args[0], _Sym)
                and (args[0].module, args[0].name) == ('numpy', 'ndarray')):
          raise UnsafeModelError('unexpected _reconstruct arguments')
        stack.append(_ArrayStub())
      elif key == ('numpy', 'dtype'):
        if not (isinstance(args, tuple) and args and isinstance(args[0], str)):
          raise UnsafeModelError('unexpected dtype arguments')
        stack.append(_DtypeStub(args[0]))
      elif key in _SCALAR:
        dt, raw = _dtype_of(args[0]), args[1]
        stack.append(np.frombuffer(raw, dtype=dt)[0])
      else:
        raise UnsafeModelError('REDUCE on {!r}'.format(fn))
    elif c == 0x62:    # BUILD
      state = stack.pop(); obj = stack[-1]
      if isinstance(obj, _DtypeStub):
        endian = state[1] if isinstance(state, tuple) and len(state) > 1 else '='
        base = np.dtype(obj.base)
        obj.value = base.newbyteorder(endian) if endian in '<>' else base
      elif isinstance(obj, _ArrayStub):
        if not (isinstance(state, tuple) and len(state) == 5):
          raise UnsafeModelError('unexpected ndarray state')
        _, shape, dt, fortran, raw = state
        dt = _dtype_of(dt)
        if isinstance(raw, list):
          raise UnsafeModelError('object arrays are not model data')
        arr = np.frombuffer(bytes(raw), dtype=dt).copy()
        obj.value = arr.reshape(shape, order='F' if fortran else 'C')
      else:
        raise UnsafeModelError('BUILD on {!r}'.format(type(obj)))
    else:
      raise UnsafeModelError('unsupported pickle opcode 0x{:02x}'.format(c))
  if len(stack) != 1:
    raise UnsafeModelError('malformed pickle stack')
  return _finish(stack[0])


def _from_npz(path):
  with np.load(path, allow_pickle=False) as z:
    model = {}
    for k in z.files:
      v = z[k]
      if v.ndim == 0:
        v = v.item()
      model[k] = v
  return model


def save_model_npz(model, path):
  np.savez_compressed(path, **{k: np.asarray(v) for k, v in model.items()})


def load_model_file(path):
  if path.endswith('.npz'):
    return _from_npz(path)
  with open(path, 'rb') as fp:
    return parse_model_pickle(fp.read())


def builtin_models():
  return sorted(f[:-4] + '.pkl' for f in os.listdir(BUILTIN_DIR) if f.endswith('.npz'))


def get_read_model(modelfile):
  """Mirror of reference `cli.get_read_model` (`mitty/cli.py:255-278`): built-in name first, else a literal path.

  Returns (read_module, model).  `read_module` is `None` for an unknown `model_class`, as in the reference.
  """
  import mitty_amd.simulation.illumina as illumina
  stem = modelfile[:-4] if modelfile.endswith('.pkl') else modelfile
  builtin = os.path.join(BUILTIN_DIR, os.path.basename(stem) + '.npz')
  if os.path.basename(stem) == stem and os.path.exists(builtin):
    model = _from_npz(builtin)
  else:
    model = load_model_file(modelfile)
  read_module = {'illumina': illumina}.get(model.get('model_class'))
  return read_module, model
