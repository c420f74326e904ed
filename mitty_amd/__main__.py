"""`python -m mitty_amd ...` = the `mitty` console command (setup.py)."""
from mitty_amd.cli import cli

if __name__ == '__main__':
  cli()
