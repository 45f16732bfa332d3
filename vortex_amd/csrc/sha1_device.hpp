// sha1_device.hpp — SHA-1 (FIPS 180-4) building blocks for gfx950 (CDNA4).
//
// One lane owns one piece: SHA-1 is a strict chain of 64-byte compressions,
// so a piece cannot be split; parallelism is across pieces (SURVEY.md §5,
// "long pieces").  The arithmetic is pure 32-bit integer VALU work:
//   rotates   -> v_alignbit_b32 (one op)
//   Ch/Par/Maj-> v_bitop3_b32   (one op; gfx950-only instruction)
//   4-way add -> 2 x v_add3_u32 (K rides in an SGPR)
//   bswap     -> v_perm_b32
// i.e. 5 VALU per round + 3 per scheduled word + 16 byte swaps ≈ 613 VALU per
// 64-byte block.  No MFMA: this is bitwise work, not a contraction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vx {

constexpr uint32_t kK0 = 0x5A827999u;
constexpr uint32_t kK1 = 0x6ED9EBA1u;
constexpr uint32_t kK2 = 0x8F1BBCDCu;
constexpr uint32_t kK3 = 0xCA62C1D6u;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) {
    return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

// v_bitop3_b32 truth tables with src0=0xF0, src1=0xCC, src2=0xAA.
#define VX_CH(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xCA)
#define VX_PAR(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0x96)
#define VX_MAJ(b, c, d) __builtin_amdgcn_bitop3_b32((b), (c), (d), 0xE8)
// a ^ b as an 8-byte VOP3 v_bitop3_b32 (same issue cost as the 4-byte VOP2
// v_xor_b32).  The message schedule's xor is the only 4-byte VALU op in the
// hot loops; as VOP2 it flipped the 8-byte alignment of every instruction
// after it, so ~1 in 4 of them straddled a 32-byte fetch boundary, and on
// gfx950 each straddle cost about one issue slot.
// -DVX_XOR2_VOP2 (A/B only): the plain 4-byte VOP2 xor.  Even with 2 or 4 waves per
// SIMD, where a VOP2 op takes its SIMD half the cycles of a VOP3 one, it was no
// faster (profiles/r02/negative/ab_xor_vop2.txt).
#ifdef VX_XOR2_VOP2
#define VX_XOR2(a, b) ((a) ^ (b))
#else
#define VX_XOR2(a, b) __builtin_amdgcn_bitop3_b32((a), (b), (b), 0x3C)
#endif

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

struct State {
    uint32_t h0, h1, h2, h3, h4;
};

__device__ __forceinline__ State iv() {
    return State{0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
}

// Compress one block; w[] holds the 16 big-endian message words and is used
// as the rolling schedule buffer (clobbered).
__device__ __forceinline__ void compress(State& s, uint32_t (&w)[16]) {
    uint32_t a = s.h0, b = s.h1, c = s.h2, d = s.h3, e = s.h4;
#pragma unroll
    for (int t = 0; t < 80; ++t) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rotl(VX_XOR2(VX_PAR(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]), w[t & 15]), 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20) {
            f = VX_CH(b, c, d);
            k = kK0;
        } else if (t < 40) {
            f = VX_PAR(b, c, d);
            k = kK1;
        } else if (t < 60) {
            f = VX_MAJ(b, c, d);
            k = kK2;
        } else {
            f = VX_PAR(b, c, d);
            k = kK3;
        }
        const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
        e = d;
        d = c;
        c = rotl(b, 30);
        b = a;
        a = tmp;
    }
    s.h0 += a;
    s.h1 += b;
    s.h2 += c;
    s.h3 += d;
    s.h4 += e;
}

// Compress the 64-byte block held little-endian in four uint4 registers.
__device__ __forceinline__ void compress_le(State& s, const uint4& q0, const uint4& q1, const uint4& q2,
                                            const uint4& q3) {
    uint32_t w[16] = {bswap(q0.x), bswap(q0.y), bswap(q0.z), bswap(q0.w), bswap(q1.x), bswap(q1.y),
                      bswap(q1.z), bswap(q1.w), bswap(q2.x), bswap(q2.y), bswap(q2.z), bswap(q2.w),
                      bswap(q3.x), bswap(q3.y), bswap(q3.z), bswap(q3.w)};
    compress(s, w);
}

// FIPS 180-4 §5.1.1 padding of the last `rem` (< 64) bytes at q, for a
// message of total_len bytes: one block when rem <= 55, else two.  Reads only
// bytes [q, q+rem): never touches memory past the piece.
__device__ __forceinline__ void finalize(State& s, const uint8_t* q, uint32_t rem, uint64_t total_len) {
    uint32_t w[16];
    const uint32_t* q32 = reinterpret_cast<const uint32_t*>(q);  // q is 4-byte aligned
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const uint32_t off = 4u * k;
        uint32_t v = 0;
        if (off + 4 <= rem) {
            v = q32[k];
        } else if (off < rem) {
            for (uint32_t j = 0; off + j < rem; ++j) v |= (uint32_t)q[off + j] << (8 * j);
        }
        if (rem >= off && rem < off + 4) v |= 0x80u << (8 * (rem - off));
        w[k] = bswap(v);
    }
    const uint32_t bits_hi = (uint32_t)((total_len * 8u) >> 32);
    const uint32_t bits_lo = (uint32_t)(total_len * 8u);
    if (rem <= 55) {
        w[14] = bits_hi;
        w[15] = bits_lo;
        compress(s, w);
    } else {
        compress(s, w);
        uint32_t z[16];
#pragma unroll
        for (int k = 0; k < 14; ++k) z[k] = 0;
        z[14] = bits_hi;
        z[15] = bits_lo;
        compress(s, z);
    }
}

}  // namespace vx
