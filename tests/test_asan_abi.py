"""Host-side AddressSanitizer run of the C-ABI ("race detection /
sanitizers"): build/asan_abi is raocp_capi.hip's host code compiled with
-fsanitize=address (device code uninstrumented; `make -C raocp-toolbox_amd asan`, run by
__graft_entry__.build()) linked with tests/asan/abi_driver.cpp, which drives every entry
point. CPU: tree validation and error paths. GPU: the whole lifecycle (create, operators,
prox steps, step size, CP runs, bench helpers, two shards with device-copy transport).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "asan_abi")


def _run(mode, timeout):
    if not os.path.exists(BIN):
        pytest.skip("build/asan_abi not built (make -C raocp-toolbox_amd asan)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([BIN, mode], capture_output=True, text=True, timeout=timeout, env=env)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and f"abi_driver {mode}: ok" in out, out[-4000:]


def test_asan_abi_validation_paths():
    _run("cpu", 120)


@pytest.mark.gpu
def test_asan_abi_full_lifecycle():
    _run("gpu", 240)
