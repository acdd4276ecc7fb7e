"""The C restatement of the reference (oracle/orc_majority.c) under the host
sanitizers (SURVEY §5 aux: race/memory checking on host code): a driver
(oracle/orc_sanitize_main.c) built with -fsanitize=address,undefined runs
rollouts on random ELL/CSR arrays and SA loops at several (d, p, c); any
out-of-bounds access or undefined behaviour aborts it.  CPU only."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def test_c_oracle_under_asan_ubsan(tmp_path):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    src = os.path.join(ROOT, "oracle", "orc_sanitize_main.c")
    exe = str(tmp_path / "orc_sanitize")
    cmd = [gcc, "-std=gnu99", "-O1", "-g", "-ffp-contract=off", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", src, "-o", exe, "-lm"]
    build = subprocess.run(cmd, capture_output=True, text=True)
    if build.returncode != 0 and "asan" in (build.stderr or "").lower():
        pytest.skip("sanitizer runtime not installed: " + build.stderr[-200:])
    assert build.returncode == 0, build.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert run.returncode == 0 and run.stdout.strip().endswith("ok"), run.stdout[-2000:] + run.stderr[-2000:]
