"""The download path at network-realistic arrival rates:
tools/native/paced_probe models vortex's event loop — pieces arrive at R GB/s
into registered pool buffers, each 1 ms turn submits what arrived, flushes
once and polls (peer_connection.rs:1145-1158, event_loop.rs:554-557).  Below
the PCIe rate the loop thread must never block in vx_submit (scope.spawn
never does) and every verdict must arrive well inside the loop's 150 ms CQE
wait (event_loop.rs:438-439); planted mismatches must come back as such."""
import json
import os
import subprocess

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

EXE = os.path.join(ROOT, "tools", "native", "paced_probe")


@pytest.fixture(scope="module")
def probe(built):
    subprocess.run(["make", "-C", os.path.dirname(EXE), "-s", "paced_probe"], check=True)
    return EXE


@pytest.mark.parametrize("plen,rate", [(262144, 4), (262144, 16), (2 << 20, 4), (16384, 2)])
def test_paced_download_loop(gpu, probe, plen, rate):
    nbuf = max(256, min(4096, (1 << 30) // plen))  # at most 1 GiB of pool buffers
    p = subprocess.run([probe, str(plen), str(rate), "0.6", "1000", str(nbuf)], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["mismatched_verdicts"] == 0 and d["pieces"] > 0
    assert d["achieved_GBps"] == pytest.approx(rate, rel=0.05)
    assert d["submit_stall_ms_per_s"] == 0.0  # the loop thread never waited for a batch
    assert d["latency_ms"]["p99"] < 150.0
    assert d["loop_ms_per_s"] < 250.0  # a quarter of the thread at most (measured: 5-70 ms/s)
