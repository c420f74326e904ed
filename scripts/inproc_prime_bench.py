"""Fresh-box A/B (DESIGN.md "the first process"): the HBM prime pass of scripts/prime_hbm.py run in THIS process
(same HIP runtime the library then uses), then bench.py's main() in the same process with the given arguments."""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'scripts'))
import prime_hbm  # noqa: E402

saved = sys.argv[1:]
sys.argv = ['prime_hbm.py', '0', '8', os.environ.get('PRIME_WRITE', '1')]
prime_hbm.main()
sys.argv = [os.path.join(REPO, 'bench.py')] + saved
runpy.run_path(os.path.join(REPO, 'bench.py'), run_name='__main__')
