"""Download-path submit-to-poll latency with and without the zero-copy slot
kernel: tests/native/loop_harness at several piece
lengths, VX_ZERO_COPY=0 (gather + hash) against 1, alternating, one JSON line
per run with the harness's p50 / p99 latency and throughput.

    python3 tools/loop_latency_ab.py [--reps 2]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--values", default="0,1", help="VX_ZERO_COPY values to alternate (anything but 0 = the default)")
    a = ap.parse_args()
    import oracle

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    cases = [(2000, 32768, 164), (600, 262144, 262144 - 16384 - 77), (97, 2097152, 1179648),
             (48, 4194304, 4194304 - 4096)]
    exe = os.path.join(ROOT, "tests", "native", "loop_harness")
    with tempfile.TemporaryDirectory() as d:
        for n, plen, last in cases:
            seed = 0x5EED00AA
            p = os.path.join(d, f"exp_{plen}.bin")
            with open(p, "wb") as f:
                f.write(oracle.pool_digest_synth(seed, 0, n, plen, last_index=n - 1, last_len=last, threads=threads))
            for rep in range(a.reps):
                for zc in a.values.split(","):
                    env = dict(os.environ, VX_ZERO_COPY=zc)
                    out = subprocess.run([exe, p, str(n), str(plen), str(last), hex(seed), "32", "4", "50"],
                                         capture_output=True, text=True, timeout=300, env=env)
                    if out.returncode != 0:
                        raise SystemExit(out.stdout + out.stderr)
                    res = json.loads(out.stdout.strip().splitlines()[-1])
                    res.pop("engine", None)
                    print(json.dumps({"zero_copy": int(zc), "rep": rep, "pieces": n, "piece_len": plen, **res}),
                          flush=True)


if __name__ == "__main__":
    main()
