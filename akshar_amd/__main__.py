"""python -m akshar_amd ... (akshar_amd/cli.py)."""
from .cli import main

main()
