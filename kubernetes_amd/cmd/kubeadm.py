"""kubeadm entry point."""
import sys

from ..kubeadm.cli import main

if __name__ == "__main__":
    sys.exit(main())
