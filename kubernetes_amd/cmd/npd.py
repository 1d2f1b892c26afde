"""node-problem-detector entry point (the `cluster/addons/node-problem-detector` DaemonSet)."""
from ..addons.npd import main

if __name__ == "__main__":
    main()
