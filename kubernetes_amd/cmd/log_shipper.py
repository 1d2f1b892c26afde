"""Node logging agent entry point (the `cluster/addons/fluentd-elasticsearch` DaemonSet)."""
from ..addons.logging import main

if __name__ == "__main__":
    main()
