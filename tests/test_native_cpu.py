"""CPU tests of host-side native code (no GPU): the pread pool behind
vx_verify_files (vortex_amd/csrc/vx_files.hpp), stressed with back-to-back
generations whose item vector is rebuilt between runs (and the pipelined
start/wait form), plain, under ThreadSanitizer and under ASan+UBSan (host
code only, as the GPU pool allows)."""
import json
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

SRC = os.path.join(ROOT, "tests", "native", "readers_stress.cpp")


@pytest.mark.parametrize("sanitize", [None, "thread", "address,undefined"])
def test_reader_pool_generations(tmp_path, sanitize):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = tmp_path / ("rs_" + (sanitize or "plain").replace(",", "_"))
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "vortex_amd", "csrc"), SRC, "-o", str(exe), "-lpthread"]
    if sanitize:
        cmd.insert(1, "-fsanitize=" + sanitize)
        if "undefined" in sanitize:
            cmd.insert(2, "-fno-sanitize-recover=undefined")
    subprocess.run(cmd, check=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    out = subprocess.run([str(exe), str(tmp_path / "scratch.bin"), "1500", "6"], capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stdout + out.stderr[-4000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["errors"] == 0
