"""kubectl entry point."""
import sys

from ..kubectl.cli import main

if __name__ == "__main__":
    sys.exit(main())
