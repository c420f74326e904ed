"""Packaging: the `mitty` console command (reference setup.py:12, `mitty = mitty.cli:cli`) bound to the MI355X
build's CLI.  The HIP library is built in-tree first (`make -C mitty_amd/csrc`, or __graft_entry__.build())."""
from setuptools import find_packages, setup

setup(
  name='mitty-mi355x',
  version='2.7.3.dev0+mi355x',
  description='Mitty generate-reads hot path on MI355X (gfx950): HIP kernels behind the reference CLI',
  packages=find_packages(include=['mitty_amd', 'mitty_amd.*']),
  package_data={'mitty_amd': ['_lib/libmitty_hip.so', 'data/readmodels/*.npz']},
  entry_points={'console_scripts': ['mitty = mitty_amd.cli:cli']},
  install_requires=['numpy', 'click'],
  python_requires='>=3.8',
)
