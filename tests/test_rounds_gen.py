"""CPU: the generated SHA-1 consumer asm (vortex_amd/csrc/sha1_consumer_asm.inc).

The split kernels' consumer runs a fixed instruction stream written by
tools/gen_sha1_rounds.py.  Checked here without a GPU:

* the 80-round stream, simulated instruction by instruction, equals the
  FIPS 180-4 compression on random states and blocks (and hashlib on "abc");
* every block body inside the consumer loop is that same stream on its word
  set, with exactly the 20 ring reads of the next block, and both the plain
  and the ragged-select consumer pass 1 + nb_wave barriers' worth of
  structure (one barrier before the loop, one per unrolled block);
* the committed header is what the generator produces now.
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import gen_sha1_rounds as g  # noqa: E402


def test_round_stream_is_fips_sha1():
    g.check()


def test_consumer_block_bodies():
    for select in (False, True):
        text = g.consumer_asm(select)
        lines = text.splitlines()
        assert sum(1 for ln in lines if ln == "s_barrier") == 1 + 6  # before the loop + one per unrolled block
        reads = [ln for ln in lines if ln.startswith("ds_read_b128")]
        bodies = 6 * (2 if select else 1)
        assert len(reads) == 20 + 20 * bodies
        offs = sorted({int(re.search(r"offset:(\d+)", r).group(1)) for r in reads})
        assert offs == sorted({s * g.SLOT_BYTES + q * g.QUAD_BYTES for s in range(3) for q in range(20)})
        assert max(offs) < 65536  # ds_read offset field
        # each unrolled block runs the verified round stream on its word set
        for wbase in (g.WA, g.WB):
            R = g.consumer_regs(wbase)
            ins, final = g.rounds(R)
            body = g.emit(ins, final, R.h, feed_forward=True)
            assert text.count(body) == (2 if select else 1) * 3, wbase
        regs = {int(m) for m in re.findall(r"\bv(\d+)\b", text)} | {
            int(a) for a, b in re.findall(r"v\[(\d+):(\d+)\]", text)}
        assert max(regs) <= 255  # architectural VGPRs only
        clob = {int(c[1:]) for c in g.consumer_clobbers(select) if re.fullmatch(r"v\d+", c)}
        assert regs <= clob


def test_committed_header_is_current(tmp_path):
    out = tmp_path / "h.inc"
    g.write_consumer_header(str(out), "burst")
    assert out.read_text() == open(os.path.join(ROOT, "vortex_amd", "csrc", "sha1_consumer_asm.inc")).read()
