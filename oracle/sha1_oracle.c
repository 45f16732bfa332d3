/*
 * oracle/sha1_oracle.c — TEST INFRASTRUCTURE ONLY (the CPU oracle).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code, and only as the checker / the timed CPU baseline.  The product path
 * (vortex_amd/) never links or calls it.
 *
 * What it restates
 * ----------------
 * The arithmetic of vortex's hashing pool lives in the third-party crate
 * `sha1` 0.11.0 (RustCrypto, Cargo.lock:2593-2601; expected digests come from
 * lava_torrent 0.11.1 via `sha1` 0.10.7, Cargo.lock:1444-1456).  Neither is
 * vendored under /root/reference, so this file restates the published
 * algorithm both crates implement: FIPS 180-4 SHA-1 (plain SHA-1, not the
 * collision-detecting sha1dc).  Call sites it stands in for:
 *   bittorrent/src/peer_comm/peer_connection.rs:1146-1149  (download verify)
 *   bittorrent/src/file_store.rs:235, 298, 302            (bulk re-verify)
 *
 * Two compression back ends, chosen at run time like `sha1` 0.11 does through
 * `cpufeatures 0.3` on x86: the SHA-NI one when the CPU has it, else scalar.
 *
 * Parity pinning: tests/test_oracle.py checks both back ends against the FIPS
 * vectors, the reference's implicit known answers (the
 * setup_test / setup_seeding_test pieces of bittorrent/src/lib.rs:169-285) and
 * hashlib-generated fixtures in tests/golden/.
 *
 * The synthetic piece generator (vxo_gen_piece) is the CPU twin of the device
 * generator in vortex_amd/csrc/vx_synth.hip; both follow the spec in DESIGN.md
 * ("Synthetic pieces").
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#if defined(__x86_64__)
#include <cpuid.h>
#include <immintrin.h>
#endif

/* ------------------------------------------------------------------ scalar */

static inline uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static inline uint32_t load_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

/* FIPS 180-4 §6.1.2 compression of `nblocks` 64-byte blocks. */
static void compress_scalar(uint32_t st[5], const uint8_t* data, size_t nblocks) {
    for (size_t blk = 0; blk < nblocks; ++blk, data += 64) {
        uint32_t w[80];
        for (int t = 0; t < 16; ++t) w[t] = load_be32(data + 4 * t);
        for (int t = 16; t < 80; ++t) w[t] = rol32(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
        for (int t = 0; t < 80; ++t) {
            uint32_t f, k;
            if (t < 20)      { f = (b & c) | (~b & d);           k = 0x5A827999u; }
            else if (t < 40) { f = b ^ c ^ d;                    k = 0x6ED9EBA1u; }
            else if (t < 60) { f = (b & c) | (b & d) | (c & d);  k = 0x8F1BBCDCu; }
            else             { f = b ^ c ^ d;                    k = 0xCA62C1D6u; }
            uint32_t tmp = rol32(a, 5) + f + e + k + w[t];
            e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
        }
        st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
    }
}

/* ----------------------------------------------------------------- SHA-NI */
#if defined(__x86_64__)
__attribute__((target("sha,sse4.1,ssse3")))
static void compress_shani(uint32_t st[5], const uint8_t* data, size_t nblocks) {
    const __m128i bswap_mask = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
    __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)st), 0x1B);
    __m128i e0 = _mm_set_epi32((int)st[4], 0, 0, 0);
    for (size_t blk = 0; blk < nblocks; ++blk, data += 64) {
        const __m128i abcd_save = abcd, e_save = e0;
        __m128i m0 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(data + 0)), bswap_mask);
        __m128i m1 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(data + 16)), bswap_mask);
        __m128i m2 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(data + 32)), bswap_mask);
        __m128i m3 = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(data + 48)), bswap_mask);
        __m128i e, prev;
        /* Quad-round q uses message quad M[q]; for q >= 4
         *   M[q] = msg2(msg1(M[q-4], M[q-3]) ^ M[q-2], M[q-1])
         * which is W[t] = rol1(W[t-3]^W[t-8]^W[t-14]^W[t-16]) four words at a time. */
#define QR(M, FN)                                   \
        e = _mm_sha1nexte_epu32(prev, M);           \
        prev = abcd;                                \
        abcd = _mm_sha1rnds4_epu32(abcd, e, FN);
#define NEXTMSG(A, B, C, D) A = _mm_sha1msg2_epu32(_mm_xor_si128(_mm_sha1msg1_epu32(A, B), C), D);
        e = _mm_add_epi32(e0, m0);
        prev = abcd;
        abcd = _mm_sha1rnds4_epu32(abcd, e, 0);          /* q0  */
        QR(m1, 0)                                         /* q1  */
        QR(m2, 0)                                         /* q2  */
        QR(m3, 0)                                         /* q3  */
        NEXTMSG(m0, m1, m2, m3) QR(m0, 0)                 /* q4  */
        NEXTMSG(m1, m2, m3, m0) QR(m1, 1)                 /* q5  */
        NEXTMSG(m2, m3, m0, m1) QR(m2, 1)
        NEXTMSG(m3, m0, m1, m2) QR(m3, 1)
        NEXTMSG(m0, m1, m2, m3) QR(m0, 1)
        NEXTMSG(m1, m2, m3, m0) QR(m1, 1)                 /* q9  */
        NEXTMSG(m2, m3, m0, m1) QR(m2, 2)                 /* q10 */
        NEXTMSG(m3, m0, m1, m2) QR(m3, 2)
        NEXTMSG(m0, m1, m2, m3) QR(m0, 2)
        NEXTMSG(m1, m2, m3, m0) QR(m1, 2)
        NEXTMSG(m2, m3, m0, m1) QR(m2, 2)                 /* q14 */
        NEXTMSG(m3, m0, m1, m2) QR(m3, 3)                 /* q15 */
        NEXTMSG(m0, m1, m2, m3) QR(m0, 3)
        NEXTMSG(m1, m2, m3, m0) QR(m1, 3)
        NEXTMSG(m2, m3, m0, m1) QR(m2, 3)
        NEXTMSG(m3, m0, m1, m2) QR(m3, 3)                 /* q19 */
#undef QR
#undef NEXTMSG
        e0 = _mm_sha1nexte_epu32(prev, e_save);
        abcd = _mm_add_epi32(abcd, abcd_save);
    }
    _mm_storeu_si128((__m128i*)st, _mm_shuffle_epi32(abcd, 0x1B));
    st[4] = (uint32_t)_mm_extract_epi32(e0, 3);
}
#endif

int vxo_has_shani(void) {
#if defined(__x86_64__)
    unsigned a, b, c, d;
    if (!__get_cpuid_count(7, 0, &a, &b, &c, &d)) return 0;
    if (!(b & (1u << 29))) return 0; /* SHA */
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & (1u << 19)) && (c & (1u << 9)); /* SSE4.1, SSSE3 */
#else
    return 0;
#endif
}

typedef void (*compress_fn)(uint32_t*, const uint8_t*, size_t);

static compress_fn pick(int backend) {
    /* backend: 0 = auto (like cpufeatures), 1 = scalar, 2 = SHA-NI */
#if defined(__x86_64__)
    if (backend == 2 || (backend == 0 && vxo_has_shani())) return compress_shani;
#endif
    (void)backend;
    return compress_scalar;
}

/* One-shot SHA-1 = Sha1::new(); update(data[..len]); finalize() (FIPS 180-4
 * §5.1.1 padding: 0x80, zeros, 64-bit big-endian bit length). */
void vxo_sha1_backend(const uint8_t* data, size_t len, uint8_t out[20], int backend) {
    compress_fn fn = pick(backend);
    uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    size_t full = len / 64;
    if (full) fn(st, data, full);
    uint8_t tail[128];
    size_t rem = len - full * 64;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, data + full * 64, rem);
    tail[rem] = 0x80;
    size_t tblocks = (rem + 9 <= 64) ? 1 : 2;
    uint64_t bits = (uint64_t)len * 8u;
    for (int i = 0; i < 8; ++i) tail[tblocks * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    fn(st, tail, tblocks);
    for (int i = 0; i < 5; ++i) {
        out[4 * i + 0] = (uint8_t)(st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(st[i] >> 8);
        out[4 * i + 3] = (uint8_t)(st[i]);
    }
}

void vxo_sha1(const uint8_t* data, size_t len, uint8_t out[20]) { vxo_sha1_backend(data, len, out, 0); }

/* Streaming form used by the multi-file re-verify restatement
 * (file_store.rs:235-302 calls hasher.update once per file segment). */
typedef struct {
    uint32_t st[5];
    uint64_t len;
    uint8_t buf[64];
    uint32_t nbuf;
    int backend;
} vxo_sha1_ctx;

size_t vxo_sha1_ctx_size(void) { return sizeof(vxo_sha1_ctx); }

void vxo_sha1_init(vxo_sha1_ctx* c, int backend) {
    static const uint32_t iv[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    memcpy(c->st, iv, sizeof iv);
    c->len = 0;
    c->nbuf = 0;
    c->backend = backend;
}

void vxo_sha1_update(vxo_sha1_ctx* c, const uint8_t* p, size_t n) {
    compress_fn fn = pick(c->backend);
    c->len += n;
    if (c->nbuf) {
        size_t take = 64 - c->nbuf < n ? 64 - c->nbuf : n;
        memcpy(c->buf + c->nbuf, p, take);
        c->nbuf += (uint32_t)take; p += take; n -= take;
        if (c->nbuf == 64) { fn(c->st, c->buf, 1); c->nbuf = 0; }
    }
    if (n >= 64) { fn(c->st, p, n / 64); p += (n / 64) * 64; n %= 64; }
    if (n) { memcpy(c->buf, p, n); c->nbuf = (uint32_t)n; }
}

void vxo_sha1_final(vxo_sha1_ctx* c, uint8_t out[20]) {
    compress_fn fn = pick(c->backend);
    uint8_t tail[128];
    memset(tail, 0, sizeof tail);
    memcpy(tail, c->buf, c->nbuf);
    tail[c->nbuf] = 0x80;
    size_t tblocks = (c->nbuf + 9 <= 64) ? 1 : 2;
    uint64_t bits = c->len * 8u;
    for (int i = 0; i < 8; ++i) tail[tblocks * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
    fn(c->st, tail, tblocks);
    for (int i = 0; i < 5; ++i) {
        out[4 * i + 0] = (uint8_t)(c->st[i] >> 24);
        out[4 * i + 1] = (uint8_t)(c->st[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->st[i] >> 8);
        out[4 * i + 3] = (uint8_t)(c->st[i]);
    }
}

/* ------------------------------------------------------ synthetic pieces */
/* Spec (DESIGN.md "Synthetic pieces"): piece p of a stream with seed s is the
 * little-endian byte image of words
 *     key  = mix64(s ^ (p * 0xD1B54A32D192ED03))
 *     w[i] = mix64(key + (i + 1) * 0x9E3779B97F4A7C15)
 * truncated to the piece length.  If corrupt_every != 0 and
 * p % corrupt_every == corrupt_every - 1, byte (p * 7919) % len is XORed with
 * 0xFF after generation (exercises the hash-mismatch branch,
 * torrent.rs:429-440). */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void vxo_gen_piece(uint64_t seed, uint64_t piece, uint32_t len, uint32_t corrupt_every, uint8_t* out) {
    uint64_t key = mix64(seed ^ (piece * 0xD1B54A32D192ED03ULL));
    uint32_t nw = len / 8;
    for (uint32_t i = 0; i < nw; ++i) {
        uint64_t w = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
        memcpy(out + 8 * (size_t)i, &w, 8); /* x86 is little-endian */
    }
    if (len % 8) {
        uint64_t w = mix64(key + (uint64_t)(nw + 1) * 0x9E3779B97F4A7C15ULL);
        memcpy(out + 8 * (size_t)nw, &w, len % 8);
    }
    if (corrupt_every && len && (piece % corrupt_every) == corrupt_every - 1)
        out[(piece * 7919u) % len] ^= 0xFF;
}

int vxo_is_corrupt(uint64_t piece, uint32_t corrupt_every) {
    return corrupt_every && (piece % corrupt_every) == corrupt_every - 1;
}
