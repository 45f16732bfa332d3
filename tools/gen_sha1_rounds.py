#!/usr/bin/env python3
"""Generate the 80 SHA-1 rounds of one 64-byte block as a gfx950 instruction
stream with a fixed issue order and register map, and check it.

Why: a lone wave (the split kernel's consumer) runs hipcc's
round code at ~4.5 cycles per VALU against a 4-cycle issue floor
(EXPERIMENTS.md, round 2), and hipcc decides both the order and the
registers.  This emits the rounds with both fixed, and `--consumer` writes the
split kernels' consumer loop (vortex_amd/csrc/sha1_consumer_asm.inc) from them.

Dataflow (FIPS 180-4 round t: T = rotl5(a) + f(b, c, d) + e + K + W[t];
e = d; d = c; c = rotl30(b); b = a; a = T).  With A_t = T of round t:
a_t = A_{t-1}, b_t = A_{t-2}, c_t = C_{t-3}, d_t = C_{t-4}, e_t = C_{t-5}
where C_s = rotl30(A_s), A_{-1} = h0, A_{-2} = h1, C_{-3} = h2, C_{-4} = h3,
C_{-5} = h4.  So f of round t+1 needs only values from round t-1 and older,
and the chain through a is two ops per round: rotl5 then the final add3.

Issue order per round t (steady state):
    X_{t+1} = e_{t+1} + K + W[t+1]         v_add3_u32 (K in an SGPR)
    R       = rotl5(A_{t-1})               v_alignbit_b32
    F_{t+1} = f(A_{t-1}, C_{t-2}, C_{t-3}) v_bitop3_b32
    C_{t-1} = rotl30(A_{t-1})              v_alignbit_b32
    A_t     = R + F_t + X_t                v_add3_u32
so every dependent pair is at least two issue slots apart and no two
alignbits are adjacent (back-to-back v_alignbit_b32 cost ~4.8 cycles each
on one wave; tools/native/valu_issue_probe.hip).

`python tools/gen_sha1_rounds.py --check` simulates the emitted stream and
compares the block's output with hashlib's SHA-1 compression.
"""
from __future__ import annotations

import argparse
import hashlib
import random
import struct
import sys

K = [0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xCA62C1D6]
FN = {0: 0xCA, 1: 0x96, 2: 0xE8, 3: 0x96}  # bitop3 tables: Ch, Parity, Maj, Parity


def kidx(t: int) -> int:
    return t // 20


class Regs:
    """Physical register map.  h: 5 state regs; W: 80 word regs; rings for
    A (3), C (5), X (2), F (2) and one temp for rotl5."""

    def __init__(self, h, w, a, c, x, f, r, k):
        self.h, self.w, self.a, self.c, self.x, self.f, self.r, self.k = h, w, a, c, x, f, r, k

    def A(self, t):  # A_t
        return self.h[0] if t == -1 else self.h[1] if t == -2 else self.a[t % len(self.a)]

    def C(self, s):  # C_s = rotl30(A_s); C_{-3..-5} = h2..h4
        if s in (-3, -4, -5):
            return self.h[-s - 1]
        return self.c[s % len(self.c)]


def default_regs(base_h=60, base_w=100, sbase=20):
    return Regs(h=[f"v{base_h + i}" for i in range(5)], w=[f"v{base_w + i}" for i in range(80)],
                a=["v65", "v66", "v67"], c=["v68", "v69", "v70", "v71", "v72"], x=["v73", "v74"],
                f=["v75", "v76"], r="v77", k=[f"s{sbase + i}" for i in range(4)])


def rounds(R: Regs):
    """The instruction list for one block (no feed-forward): tuples
    (op, dst, srcs..., imm)."""
    ins = []
    add3k = lambda d, e, t: ins.append(("add3", d, e, R.k[kidx(t)], R.w[t]))
    # prologue: C_{-2}, F_0, X_0 (C_{-1} comes in round 0)
    ins.append(("alignbit", R.C(-2), R.A(-2), 2))
    ins.append(("bitop3", R.f[0], R.A(-2), R.C(-3), R.C(-4), FN[0]))
    add3k(R.x[0], R.C(-5), 0)
    for t in range(80):
        if t + 1 < 80:
            add3k(R.x[(t + 1) % 2], R.C(t - 4), t + 1)                       # X_{t+1}: e_{t+1} = C_{t-4}
        ins.append(("alignbit", R.r, R.A(t - 1), 27))                          # rotl5(a_t)
        if t + 1 < 80:
            ins.append(("bitop3", R.f[(t + 1) % 2], R.A(t - 1), R.C(t - 2), R.C(t - 3), FN[kidx(t + 1)]))
        if t < 79:
            ins.append(("alignbit", R.C(t - 1), R.A(t - 1), 2))                # C_{t-1} = rotl30(A_{t-1})
        ins.append(("add3", R.A(t), R.r, R.f[t % 2], R.x[t % 2]))              # A_t
    # after round 79: a = A_79, b = A_78, c = C_77, d = C_76, e = C_75
    final = [R.A(79), R.A(78), R.C(77), R.C(76), R.C(75)]
    return ins, final


def emit(ins, final, h, feed_forward=True) -> str:
    out = []
    for i in ins:
        if i[0] == "add3":
            out.append(f"v_add3_u32 {i[1]}, {i[2]}, {i[3]}, {i[4]}")
        elif i[0] == "alignbit":
            out.append(f"v_alignbit_b32 {i[1]}, {i[2]}, {i[2]}, {i[3]}")  # rotr by i[3] = rotl by 32 - i[3]
        elif i[0] == "bitop3":
            out.append(f"v_bitop3_b32 {i[1]}, {i[2]}, {i[3]}, {i[4]} bitop3:0x{i[5]:02x}")
    if feed_forward:
        for hr, fr in zip(h, final):
            out.append(f"v_add_u32_e64 {hr}, {hr}, {fr}")
    return "\n".join(out)


# ---- the split kernel's consumer loop -------------------
SLOT_BYTES = 20 * 64 * 16   # RingLds<3>: [slot][20 quads][64 lanes] of uint4
QUAD_BYTES = 64 * 16
H0, SAVE0, WA, WB = 64, 82, 96, 176  # state v64-68, rings v69-81, saved state v82-86, word sets


def consumer_regs(wbase: int) -> Regs:
    return Regs(h=[f"v{H0 + i}" for i in range(5)], w=[f"v{wbase + i}" for i in range(80)],
                a=["v69", "v70", "v71"], c=["v72", "v73", "v74", "v75", "v76"], x=["v77", "v78"],
                f=["v79", "v80"], r="v81", k=["s20", "s21", "s22", "s23"])


def _read(dst_base: int, q: int, slot: int) -> str:
    """ds_read of quad q of ring slot `slot`, addressed from %5 (lds.w[0][0][lane])."""
    return f"ds_read_b128 v[{dst_base + 4 * q}:{dst_base + 4 * q + 3}], %5 offset:{slot * SLOT_BYTES + q * QUAD_BYTES}"


def _block(R: Regs, next_slot: int, next_base: int):
    """One block: the next block's 20 ring reads into next_base (burst), then
    the 80 rounds + feed-forward on R's word registers, then lgkmcnt(0)."""
    ins, final = rounds(R)
    out = [_read(next_base, q, next_slot) for q in range(20)]
    out += emit(ins, final, R.h, feed_forward=False).splitlines()
    out += [f"v_add_u32_e64 {h}, {h}, {f}" for h, f in zip(R.h, final)]
    return out + ["s_waitcnt lgkmcnt(0)", "s_nop 0"]


def consumer_asm(select: bool) -> str:
    """The whole consumer of sha1_*split_kernel as one asm body.  Operands:
    %0-%4 state h0-h4 ("+v"), %5 LDS byte address of lds.w[0][0][lane] ("v"),
    %6 nb_wave ("s"), %7 b1 ("s"), %8 the lane's nb ("v"; used only when
    `select`).

    Barriers: none when nb_wave == 0, else one before block 0 and one after
    every block (1 + nb_wave, matching the producer's publish / producer_done).
    Ring reads of block b+1 (slot (b+1) % 3): all 20 at the top of block b into
    the other of two word sets, lgkmcnt(0) at its end ("burst": 3-7 % faster
    than hipcc's consumer of the same form; a per-quad refill was 1.5-3.5 %
    slower and one read per round 5-9 % slower, profiles/r02/consumer_asm/;
    the 6-slot ring and an LDS flag handshake were no faster, EXPERIMENTS.md).
    Blocks b >= b1 (ragged phase 2, `select`) keep the new state only in
    lanes with b < nb (v_cndmask on v_cmp b < nb).  Hot-path instructions are
    8 bytes and scalar ones come in pairs, so bodies stay 8-byte aligned
    (DESIGN.md §3.6)."""
    L = [f"v_mov_b32_e64 v{H0 + i}, %{i}" for i in range(5)]
    L += ["s_mov_b32 s20, 0x5a827999", "s_mov_b32 s21, 0x6ed9eba1", "s_mov_b32 s22, 0x8f1bbcdc",
          "s_mov_b32 s23, 0xca62c1d6", "s_mov_b32 s24, 0", f"s_mov_b32 s25, {SLOT_BYTES}",
          "s_cmp_eq_u32 %6, 0", "s_cbranch_scc1 .Lvx_end%=", "s_barrier"]
    L += [_read(WA, q, 0) for q in range(20)]
    L += ["s_waitcnt lgkmcnt(0)", "s_nop 0", ".p2align 5", ".Lvx_loop%=:"]
    for k in range(6):  # slots cycle by 3, word sets by 2
        cur, nxt = (WA, WB) if k % 2 == 0 else (WB, WA)
        body = _block(consumer_regs(cur), (k + 1) % 3, nxt)
        if select:
            L += ["s_cmp_lt_u32 s24, %7", f"s_cbranch_scc0 .Lvx_sel{k}_%=", ".p2align 3"]
            L += body
            L += [f"s_branch .Lvx_done{k}_%=", "s_nop 0", ".p2align 3", f".Lvx_sel{k}_%=:"]
            L += [f"v_mov_b32_e64 v{SAVE0 + i}, v{H0 + i}" for i in range(5)]
            L += body
            L += ["v_cmp_lt_u32_e64 vcc, s24, %8"]
            L += [f"v_cndmask_b32_e64 v{H0 + i}, v{SAVE0 + i}, v{H0 + i}, vcc" for i in range(5)]
            L += [".p2align 3", f".Lvx_done{k}_%=:"]
        else:
            L += body
        L += ["s_barrier", "s_add_u32 s24, s24, 1", "s_cmp_ge_u32 s24, %6", "s_cbranch_scc1 .Lvx_end%=",
              ".p2align 3"]
    L += ["s_branch .Lvx_loop%=", ".Lvx_end%=:", "s_waitcnt lgkmcnt(0)"]
    L += [f"v_mov_b32_e64 %{i}, v{H0 + i}" for i in range(5)]
    return "\n".join(L)


def consumer_clobbers(select: bool):
    v = [f"v{i}" for i in range(H0, SAVE0 + 5 if select else SAVE0)]
    v += [f"v{i}" for i in range(WA, WB + 80)]
    # s_cmp_* / s_add_u32 in the loop control write SCC: name it, so the compiler
    # never keeps a compare live in SCC across the asm body
    return v + ["s20", "s21", "s22", "s23", "s24", "s25", "vcc", "scc"]


def write_consumer_header(path: str, mode: str = "burst") -> None:
    with open(path, "w") as f:
        f.write("// GENERATED by tools/gen_sha1_rounds.py --consumer; do not edit.\n"
                "// The split kernels' consumer loop (ring of 3 LDS slots) as one asm body:\n"
                "// fixed issue order and registers for the 80 SHA-1 rounds (DESIGN.md §3.2).\n"
                "// Checked by tests/test_rounds_gen.py (stream simulated against FIPS 180-4,\n"
                f"// header up to date).  Ring reads: {mode}.\n#pragma once\n\n")
        for name, sel in (("VX_CONSUMER_ASM", False), ("VX_CONSUMER_SELECT_ASM", True)):
            f.write(f"#define {name} \\\n")
            for line in consumer_asm(sel).splitlines():
                f.write(f'    "{line}\\n" \\\n')
            f.write('    ""\n')
            f.write(f"#define {name}_CLOBBERS " + ", ".join(f'"{r}"' for r in consumer_clobbers(sel)) + "\n\n")


# ---- simulation (the --check) -------------------------------------------
M = 0xFFFFFFFF


def rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & M


def bitop3(a, b, c, table):
    r = 0
    for bit in range(32):
        idx = (((a >> bit) & 1) << 2) | (((b >> bit) & 1) << 1) | ((c >> bit) & 1)
        r |= ((table >> idx) & 1) << bit
    return r


def simulate(text: str, regs: dict) -> dict:
    for line in text.splitlines():
        op, rest = line.split(None, 1)
        args = [a.strip() for a in rest.replace(" bitop3:", ", bitop3:").split(",")]
        if op == "v_add3_u32":
            regs[args[0]] = (regs[args[1]] + regs[args[2]] + regs[args[3]]) & M
        elif op == "v_alignbit_b32":
            s = int(args[3])
            x = (regs[args[1]] << 32) | regs[args[2]]
            regs[args[0]] = (x >> s) & M
        elif op == "v_bitop3_b32":
            regs[args[0]] = bitop3(regs[args[1]], regs[args[2]], regs[args[3]], int(args[4].split(":")[1], 16))
        elif op == "v_add_u32_e64":
            regs[args[0]] = (regs[args[1]] + regs[args[2]]) & M
        else:
            raise ValueError(op)
    return regs


def sha1_compress_ref(h, block):
    """One FIPS 180-4 compression in plain Python (checked against hashlib below)."""
    w = list(struct.unpack(">16I", block))
    for t in range(16, 80):
        w.append(rotl(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1))
    a, b, c, d, e = h
    for t in range(80):
        if t < 20:
            f = (b & c) | (~b & d)
        elif t < 40 or t >= 60:
            f = b ^ c ^ d
        else:
            f = (b & c) | (b & d) | (c & d)
        a, b, c, d, e = (rotl(a, 5) + (f & M) + e + K[t // 20] + w[t]) & M, a, rotl(b, 30), c, d
    return [(x + y) & M for x, y in zip(h, (a, b, c, d, e))], w


def check() -> None:
    iv = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
    # the reference compression agrees with hashlib on a padded one-block message
    msg = b"abc"
    blk = msg + b"\x80" + b"\0" * (55 - len(msg)) + struct.pack(">Q", 8 * len(msg))
    out, _ = sha1_compress_ref(iv, blk)
    assert struct.pack(">5I", *out) == hashlib.sha1(msg).digest()
    R = default_regs()
    ins, final = rounds(R)
    text = emit(ins, final, R.h)
    rng = random.Random(1)
    for trial in range(20):
        h = iv if trial == 0 else [rng.getrandbits(32) for _ in range(5)]
        block = blk if trial == 0 else bytes(rng.getrandbits(8) for _ in range(64))
        want, w = sha1_compress_ref(h, block)
        regs = {r: rng.getrandbits(32) for r in R.a + R.c + R.x + R.f + [R.r]}
        regs.update({R.h[i]: h[i] for i in range(5)})
        regs.update({R.w[t]: w[t] for t in range(80)})
        regs.update({R.k[i]: K[i] for i in range(4)})
        got = simulate(text, regs)
        assert [got[r] for r in R.h] == want, trial
    n = len(ins)
    assert n == 3 + 80 * 5 - 3, n  # prologue 3, 5 per round minus the three skipped in round 79
    print(f"ok: {n} round instructions + 5 feed-forward, bit-exact vs FIPS 180-4 on 20 blocks", file=sys.stderr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--emit", action="store_true", help="print the asm body (default registers)")
    ap.add_argument("--consumer", help="write the split kernels' consumer asm header")
    a = ap.parse_args()
    if a.check:
        check()
    if a.emit:
        R = default_regs()
        print(emit(*rounds(R), R.h))
    if a.consumer:
        write_consumer_header(a.consumer)


if __name__ == "__main__":
    main()
