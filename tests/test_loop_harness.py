"""GPU: vortex's download-path control flow (subpiece assembly into registered
pool buffers → submit on completion → drain once per loop turn → re-request on
mismatch) driven through the C ABI by tests/native/loop_harness.cpp."""
import json
import os
import subprocess

import pytest

import oracle
from conftest import ROOT

pytestmark = pytest.mark.gpu
THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.mark.parametrize("n,plen,last", [(600, 262144, 262144 - 16384 - 77), (97, 2097152, 1179648),
                                         (2000, 32768, 164)])
def test_download_loop(built, gpu, tmp_path, n, plen, last):
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "native"), "-s"], check=True)
    seed = 0x5EED00AA
    exp = oracle.pool_digest_synth(seed, 0, n, plen, last_index=n - 1, last_len=last, threads=THREADS)
    p = tmp_path / "expected.bin"
    p.write_bytes(exp)
    out = subprocess.run([os.path.join(ROOT, "tests", "native", "loop_harness"), str(p), str(n), str(plen),
                          str(last), hex(seed), "32", "4", "50"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(res))
    corrupted = sum(1 for i in range(n) if i % 50 == 25)
    assert res["wrong"] == 0
    assert res["rejected"] == corrupted
    assert res["hashed"] == n + corrupted
    # the engine's own counters (vx_get_stats) agree with the loop's bookkeeping
    eng = res["engine"]
    assert eng["pieces_completed"] == res["hashed"] and eng["pieces_mismatched"] == res["rejected"]
    assert eng["bytes_completed"] == n * plen - (plen - last) + sum(
        plen if i != n - 1 else last for i in range(n) if i % 50 == 25)
    assert eng["batches"] >= 1


@pytest.mark.parametrize("fail_submit_every,fail_launch_after", [(37, -1), (0, 3), (29, 5)])
def test_download_loop_with_faults(built, gpu, tmp_path, fail_submit_every, fail_launch_after):
    """INTEGRATION.md's call sites under injected faults, in C++: refused
    submits go to vortex's own pool (the CPU restatement, results over a
    channel), and after a device failure the loop drains what finished,
    destroys the context and hands every unfinished piece to the pool, which
    hashes everything after it.  Every delivery gets exactly one verdict and
    the download still completes bit-exactly."""
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "native"), "-s"], check=True)
    n, plen, last, seed = 600, 262144, 262144 - 16384 - 77, 0x5EED00AB
    exp = oracle.pool_digest_synth(seed, 0, n, plen, last_index=n - 1, last_len=last, threads=THREADS)
    p = tmp_path / "expected.bin"
    p.write_bytes(exp)
    out = subprocess.run([os.path.join(ROOT, "tests", "native", "loop_harness"), str(p), str(n), str(plen),
                          str(last), hex(seed), "32", "4", "50", str(fail_submit_every), str(fail_launch_after)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    res = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(res))
    corrupted = sum(1 for i in range(n) if i % 50 == 25)
    assert res["wrong"] == 0 and res["rejected"] == corrupted and res["hashed"] == n + corrupted
    f = res["faults"]
    if fail_submit_every:
        assert f["refused"] > 0 and f["cpu_hashed"] >= f["refused"]
    if fail_launch_after >= 0:
        assert f["gpu_dead"] == 1 and f["cpu_hashed"] > 0
    else:
        assert f["gpu_dead"] == 0 and f["recovered"] == 0
