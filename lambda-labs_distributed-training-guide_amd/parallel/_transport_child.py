"""Entry point of the transport-calibration child job (parallel/transport.py `resolve_isolated`):
`torchrun --nproc-per-node W _transport_child.py '<spec json>'`."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import dtg  # noqa: E402,F401  (registers the package)
from dtg.parallel.transport import child_main  # noqa: E402

if __name__ == "__main__":
    sys.exit(child_main(sys.argv[1:]))
