"""Import shim: tests use make_golden's record digest without re-running it."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
from make_golden import rec_digest  # noqa: E402,F401
