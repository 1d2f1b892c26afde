"""e2e runner: `python -m kubernetes_amd.e2e --server URL [--focus RE] [--skip RE]`."""
import argparse
import asyncio
import sys

from . import specs, specs_common, specs_more, specs_storage  # noqa: F401 - registers the specs
from .framework import run_specs


def main(argv=None):
    ap = argparse.ArgumentParser("e2e")
    ap.add_argument("--server", default="http://127.0.0.1:8080")
    ap.add_argument("--token", default=None)
    ap.add_argument("--focus", default=None, help="regex over spec names, e.g. Conformance")
    ap.add_argument("--skip", default=None, help="regex, e.g. 'Feature:GPU'")
    ap.add_argument("--timeout", type=float, default=180.0)
    a = ap.parse_args(argv)
    results = asyncio.run(run_specs(a.server, a.focus, a.skip, a.token, timeout=a.timeout))
    failed = [r for r in results if not r.ok]
    skipped = sum(r.skipped for r in results)
    print(f"\nRan {len(results)} specs: {len(results) - len(failed) - skipped} passed, {len(failed)} failed, "
          f"{skipped} skipped")
    for r in failed:
        print(f"--- {r.name}\n{r.error}")
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
