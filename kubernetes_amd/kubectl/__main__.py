"""`python -m kubernetes_amd.kubectl` entry point."""
import sys

from .cli import main

sys.exit(main())
