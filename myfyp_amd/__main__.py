"""``python -m myfyp_amd`` → CLI."""

from myfyp_amd.cli import main

main()
