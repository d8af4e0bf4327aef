"""Host-side AddressSanitizer run of the C ABI (SURVEY.md §5 aux: an ASan host build of the C-ABI).

`make asan` builds tools/asan/nst_asan_driver: the C-ABI host translation units compiled with -fsanitize=address
on the host side only (GPU sanitizers are not available), linked with the normal kernels.  The driver creates a
handle of every architecture in every compute dtype from the synthetic checkpoints, plans, sizes the workspace,
runs forwards on ragged frames, calls the Gram entry point and the error paths, and destroys everything; any
heap overflow / use-after-free / double free in that host code aborts it with an ASan report."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
DRIVER = os.path.join(REPO, "tools", "asan", "nst_asan_driver")


def test_c_abi_under_host_asan(tmp_path):
    if not os.path.exists(DRIVER):
        pytest.skip("tools/asan/nst_asan_driver not built (make asan)")
    sys.path.insert(0, os.path.join(REPO, "tools", "asan"))
    import make_params
    paths = make_params.main(str(tmp_path))
    env = dict(os.environ)
    # the pool preloads a small library of its own, so ASan cannot be first in the link order; leak checking
    # would report the HIP runtime's process-lifetime allocations
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=0:abort_on_error=1"
    r = subprocess.run([DRIVER] + paths, env=env, capture_output=True, text=True, timeout=240)
    print(r.stdout[-2000:], r.stderr[-4000:])
    assert "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    assert r.stdout.strip().endswith("ok (0 failures)")
