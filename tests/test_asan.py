"""Host AddressSanitizer + UBSan runs (SURVEY §5 race/sanitizer row): the native
search (mcts_engine.cpp, whole) and the host side of the policy/value C-ABI
(pv_capi.hip with -Xarch_host -fsanitize=address) driven through their C-ABIs by
csrc/asan/*.cpp.  Any sanitizer report fails the test.  CPU only (no kernel runs)."""
import os
import subprocess

import pytest

from conftest import PKG

CSRC = os.path.join(PKG, "csrc")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-C", CSRC, "asan", "-j4"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return os.path.join(CSRC, "build_asan")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("driver", ["asan_mcts", "asan_pv"])
def test_sanitized_driver(built, driver):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(built, driver)], capture_output=True, text=True, timeout=240, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "runtime error" not in out and "AddressSanitizer" not in out and "LeakSanitizer" not in out, out[-3000:]
    assert f"{driver}: ok" in out
