"""Dev diagnostics: run a case with every fused local-apply call cross-checked against the GEMM plan."""
import os
import sys

os.environ["TTIPM_CHECK_FUSED"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402


class Stop(Exception):
    pass


def cb(it):
    if it >= int(sys.argv[5]):
        raise Stop


cfg = yaml.safe_load(open(os.path.join("configs", sys.argv[2] + ".yaml")))
try:
    run_and_record(sys.argv[1], cfg, int(sys.argv[3]), int(sys.argv[4]), verbose=False, iter_callback=cb)
except Stop:
    pass
errs = sorted(D.CHECK_LOG, key=lambda e: -e[-1])
print("checked", len(errs), "max err", errs[0][-1] if errs else None)
for e in errs[:15]:
    print(e)
