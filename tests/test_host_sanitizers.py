"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only; GPU sanitizers are not available
on the pool): the MT19937 restatement and its jump-ahead (bc_mpc_amd/csrc/mt19937.cpp, mt_jump.cpp) built
with g++ -fsanitize=address,undefined from the library's own sources and self-checked
(tests/cpp/mt_host_check.cpp: one-pass vs staged draw, threaded jump-ahead vs serial draw, mt_state_at vs
stepping, A = 1..16, odd stream positions)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_mt_host_code_clean_under_asan_ubsan(tmp_path):
    src = os.path.join(REPO, "bc_mpc_amd", "csrc")
    exe = str(tmp_path / "mt_host_check")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-I", src, os.path.join(REPO, "tests", "cpp", "mt_host_check.cpp"),
           os.path.join(src, "mt19937.cpp"), os.path.join(src, "mt_jump.cpp"), "-o", exe, "-lpthread"]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().startswith("ok")
