// gs_ed25519.h -- SHA3-512 and ed25519 arithmetic of gs_verify.hip (see
// there for what is restated from where).  Header-only so that the same source
// compiles for the GPU kernels (ED_DEV = __device__, constants in device
// memory) and, in a host test build (ED_HOST_TEST), for the CPU check of the
// arithmetic against oracle/ed25519_sha3.py (tests/test_ed25519_host.py).
#pragma once
#include <stdint.h>

#ifdef ED_HOST_TEST
#define ED_DEV inline
#define ED_CONST static const
#else
#include <hip/hip_runtime.h>
#define ED_DEV __device__ __forceinline__
#define ED_CONST __device__ const
#endif

namespace gs {
namespace ed {

typedef unsigned long long u64;


// ------------------------------------------------------------ SHA3-512
constexpr uint32_t kRate = 72;  // bytes

ED_CONST u64 kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

ED_DEV u64 rotl(u64 v, uint32_t r) { return r ? (v << r) | (v >> (64u - r)) : v; }

// Keccak-f[1600] on the 5x5 lanes A[x + 5 y].
ED_DEV void keccak_f(u64 (&A)[25]) {
    // rho offsets of lane (x, y), and pi: B[y, 2x + 3y] = rot(A[x, y])
    constexpr uint32_t rho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                                  25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
    for (uint32_t round = 0; round < 24; ++round) {
        u64 C[5], B[25];
#pragma unroll
        for (int x = 0; x < 5; ++x) C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            const u64 d = C[(x + 4) % 5] ^ rotl(C[(x + 1) % 5], 1);
#pragma unroll
            for (int y = 0; y < 5; ++y) A[x + 5 * y] ^= d;
        }
#pragma unroll
        for (int x = 0; x < 5; ++x)
#pragma unroll
            for (int y = 0; y < 5; ++y) B[y + 5 * ((2 * x + 3 * y) % 5)] = rotl(A[x + 5 * y], rho[x + 5 * y]);
#pragma unroll
        for (int y = 0; y < 5; ++y)
#pragma unroll
            for (int x = 0; x < 5; ++x)
                A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
        A[0] ^= kKeccakRC[round];
    }
}

// SHA3-512 of the concatenation of up to three byte strings (one lane).
struct Pieces {
    const uint8_t *p[3];
    uint32_t n[3];
};
ED_DEV void sha3_512(const Pieces &in, uint8_t out[64]) {
    u64 A[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) A[i] = 0;
    uint32_t pos = 0;  // bytes absorbed into the current block
    for (int k = 0; k < 3; ++k) {
        for (uint32_t i = 0; i < in.n[k]; ++i) {
            A[pos >> 3] ^= (u64)in.p[k][i] << (8u * (pos & 7u));
            if (++pos == kRate) {
                keccak_f(A);
                pos = 0;
            }
        }
    }
    A[pos >> 3] ^= (u64)0x06 << (8u * (pos & 7u));
    A[(kRate - 1) >> 3] ^= (u64)0x80 << (8u * ((kRate - 1) & 7u));
    keccak_f(A);
    for (int i = 0; i < 64; ++i) out[i] = (uint8_t)(A[i >> 3] >> (8 * (i & 7)));
}

// ------------------------------------------------------------ GF(2^255 - 19)
struct Fe {
    uint32_t v[8];
};

ED_DEV Fe fe_from(uint32_t x) {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = 0;
    r.v[0] = x;
    return r;
}

// r = a + 38 * carry folded in, while carries come out
ED_DEV void fe_fold(Fe &r, uint32_t carry) {
    while (carry) {
        u64 t = (u64)r.v[0] + 38ull * carry;
        r.v[0] = (uint32_t)t;
        t >>= 32;
        for (int i = 1; i < 8; ++i) {
            t += r.v[i];
            r.v[i] = (uint32_t)t;
            t >>= 32;
        }
        carry = (uint32_t)t;
    }
}

ED_DEV Fe fe_add(const Fe &a, const Fe &b) {
    Fe r;
    u64 t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        t += (u64)a.v[i] + b.v[i];
        r.v[i] = (uint32_t)t;
        t >>= 32;
    }
    fe_fold(r, (uint32_t)t);
    return r;
}

// a - b: a wrapped result r = a - b + 2^256 stands for r - 38 (2^256 = 38 mod p)
ED_DEV Fe fe_sub(const Fe &a, const Fe &b) {
    Fe r;
    int64_t t = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        t += (int64_t)a.v[i] - (int64_t)b.v[i];
        r.v[i] = (uint32_t)t;
        t >>= 32;  // arithmetic: -1 on a borrow
    }
    uint32_t borrow = t ? 1u : 0u;
    while (borrow) {  // subtract 38 per wrap (at most twice)
        int64_t s = (int64_t)r.v[0] - 38;
        r.v[0] = (uint32_t)s;
        s >>= 32;
        for (int i = 1; i < 8 && s; ++i) {
            s += r.v[i];
            r.v[i] = (uint32_t)s;
            s >>= 32;
        }
        borrow = s ? 1u : 0u;
    }
    return r;
}

ED_DEV Fe fe_mul(const Fe &a, const Fe &b) {
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u64 c = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            c += (u64)a.v[i] * b.v[j] + w[i + j];
            w[i + j] = (uint32_t)c;
            c >>= 32;
        }
        w[i + 8] = (uint32_t)c;
    }
    // fold the high half: w_lo + 38 w_hi
    Fe r;
    u64 c = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        c += (u64)w[i] + 38ull * w[i + 8];
        r.v[i] = (uint32_t)c;
        c >>= 32;
    }
    fe_fold(r, (uint32_t)c);
    return r;
}

ED_DEV Fe fe_sq(const Fe &a) { return fe_mul(a, a); }

// the value in [0, p)
ED_DEV Fe fe_canon(const Fe &a) {
    Fe r = a;
    for (int k = 0; k < 2; ++k) {
        // p = 2^255 - 19: r >= p iff r + 19 >= 2^255
        u64 t = (u64)r.v[0] + 19u;
        uint32_t s[8];
        s[0] = (uint32_t)t;
        t >>= 32;
        for (int i = 1; i < 8; ++i) {
            t += r.v[i];
            s[i] = (uint32_t)t;
            t >>= 32;
        }
        if (t == 0 && (s[7] >> 31) == 0) break;  // r + 19 < 2^255
        // r - p = r + 19 - 2^255 (and a carry out of 2^256 cannot happen twice)
        s[7] &= 0x7FFFFFFFu;
        for (int i = 0; i < 8; ++i) r.v[i] = s[i];
        if (t) r.v[7] += 0x80000000u;  // (r + 19 >= 2^256: r - p = s + 2^255)
    }
    return r;
}

ED_DEV bool fe_eq(const Fe &a, const Fe &b) {
    const Fe x = fe_canon(a), y = fe_canon(b);
    uint32_t d = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d |= x.v[i] ^ y.v[i];
    return d == 0;
}

ED_DEV bool fe_is_zero(const Fe &a) { return fe_eq(a, fe_from(0)); }

// a^e for an exponent given by its 8 limbs (square and multiply, MSB first)
ED_DEV Fe fe_pow(const Fe &a, const uint32_t (&e)[8]) {
    Fe r = fe_from(1);
    for (int i = 255; i >= 0; --i) {
        r = fe_sq(r);
        if ((e[i >> 5] >> (i & 31)) & 1u) r = fe_mul(r, a);
    }
    return r;
}

// p - 2 and (p - 5) / 8 = 2^252 - 3
ED_CONST uint32_t kPm2[8] = {0xFFFFFFEBu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                     0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
ED_CONST uint32_t kPm5d8[8] = {0xFFFFFFFDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                       0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x0FFFFFFFu};

ED_DEV Fe fe_inv(const Fe &a) {
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = kPm2[i];
    return fe_pow(a, e);
}

ED_DEV Fe fe_load(const uint8_t *b) {  // 32 little-endian bytes
    Fe r;
    for (int i = 0; i < 8; ++i)
        r.v[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
                 ((uint32_t)b[4 * i + 3] << 24);
    return r;
}

// d = -121665 / 121666 and 2d, sqrt(-1) = 2^((p-1)/4), the base point B
ED_CONST uint32_t kD[8] = {0x135978A3u, 0x75EB4DCAu, 0x4141D8ABu, 0x00700A4Du,
                                   0x7779E898u, 0x8CC74079u, 0x2B6FFE73u, 0x52036CEEu};
ED_CONST uint32_t kD2[8] = {0x26B2F159u, 0xEBD69B94u, 0x8283B156u, 0x00E0149Au,
                                    0xEEF3D130u, 0x198E80F2u, 0x56DFFCE7u, 0x2406D9DCu};
ED_CONST uint32_t kSqrtM1[8] = {0x4A0EA0B0u, 0xC4EE1B27u, 0xAD2FE478u, 0x2F431806u,
                                        0x3DFBD7A7u, 0x2B4D0099u, 0x4FC1DF0Bu, 0x2B832480u};
ED_CONST uint32_t kBx[8] = {0x8F25D51Au, 0xC9562D60u, 0x9525A7B2u, 0x692CC760u,
                                    0xFDD6DC5Cu, 0xC0A4E231u, 0xCD6E53FEu, 0x216936D3u};
ED_CONST uint32_t kBy[8] = {0x66666658u, 0x66666666u, 0x66666666u, 0x66666666u,
                                    0x66666666u, 0x66666666u, 0x66666666u, 0x66666666u};

ED_DEV Fe fe_const(const uint32_t (&c)[8]) {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = c[i];
    return r;
}

// ------------------------------------------------------------ edwards25519
struct Pt {
    Fe X, Y, Z, T;
};

ED_DEV Pt pt_zero() { return Pt{fe_from(0), fe_from(1), fe_from(1), fe_from(0)}; }

ED_DEV Pt pt_add(const Pt &p, const Pt &q) {  // RFC 8032 5.1.4, a = -1
    const Fe a = fe_mul(fe_sub(p.Y, p.X), fe_sub(q.Y, q.X));
    const Fe b = fe_mul(fe_add(p.Y, p.X), fe_add(q.Y, q.X));
    const Fe c = fe_mul(fe_mul(p.T, q.T), fe_const(kD2));
    const Fe z = fe_mul(p.Z, q.Z);
    const Fe d = fe_add(z, z);
    const Fe e = fe_sub(b, a), f = fe_sub(d, c), g = fe_add(d, c), h = fe_add(b, a);
    return Pt{fe_mul(e, f), fe_mul(g, h), fe_mul(f, g), fe_mul(e, h)};
}

ED_DEV Pt pt_neg(const Pt &p) { return Pt{fe_sub(fe_from(0), p.X), p.Y, p.Z, fe_sub(fe_from(0), p.T)}; }

ED_DEV Pt pt_base() {
    const Fe x = fe_const(kBx), y = fe_const(kBy);
    return Pt{x, y, fe_from(1), fe_mul(x, y)};
}

ED_DEV void pt_encode(const Pt &p, uint8_t out[32]) {
    const Fe zi = fe_inv(p.Z);
    const Fe x = fe_canon(fe_mul(p.X, zi)), y = fe_canon(fe_mul(p.Y, zi));
    for (int i = 0; i < 32; ++i) out[i] = (uint8_t)(y.v[i >> 2] >> (8 * (i & 3)));
    out[31] |= (uint8_t)((x.v[0] & 1u) << 7);
}

// curve25519-dalek 0.x CompressedEdwardsY::decompress: y from the low 255
// bits (reduced mod p), x^2 = (y^2 - 1) / (d y^2 + 1), x with the sign bit
ED_DEV bool pt_decode(const uint8_t in[32], Pt &p) {
    Fe y = fe_load(in);
    const uint32_t sign = y.v[7] >> 31;
    y.v[7] &= 0x7FFFFFFFu;
    y = fe_canon(y);
    const Fe y2 = fe_sq(y);
    const Fe u = fe_sub(y2, fe_from(1));
    const Fe v = fe_add(fe_mul(y2, fe_const(kD)), fe_from(1));
    // x = u v^3 (u v^7)^((p - 5) / 8)
    const Fe v3 = fe_mul(fe_sq(v), v);
    const Fe v7 = fe_mul(fe_sq(v3), v);
    uint32_t e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = kPm5d8[i];
    Fe x = fe_mul(fe_mul(u, v3), fe_pow(fe_mul(u, v7), e));
    const Fe vx2 = fe_mul(v, fe_sq(x));
    if (!fe_eq(vx2, u)) {
        if (!fe_eq(vx2, fe_sub(fe_from(0), u))) return false;
        x = fe_mul(x, fe_const(kSqrtM1));
    }
    x = fe_canon(x);
    if ((x.v[0] & 1u) != sign) x = fe_canon(fe_sub(fe_from(0), x));
    p = Pt{x, y, fe_from(1), fe_mul(x, y)};
    return true;
}

// [a]P + [b]Q, a and b as 8 little-endian 32-bit limbs (Straus, MSB first)
ED_DEV Pt pt_mul2(const uint32_t (&a)[8], const Pt &P, const uint32_t (&b)[8], const Pt &Q) {
    const Pt PQ = pt_add(P, Q);
    Pt r = pt_zero();
    for (int i = 255; i >= 0; --i) {
        r = pt_add(r, r);
        const uint32_t sa = (a[i >> 5] >> (i & 31)) & 1u, sb = (b[i >> 5] >> (i & 31)) & 1u;
        if (sa && sb) r = pt_add(r, PQ);
        else if (sa) r = pt_add(r, P);
        else if (sb) r = pt_add(r, Q);
    }
    return r;
}

// ------------------------------------------------------------ scalars mod L
// L = 2^252 + 27742317777372353535851937790883648493; mu = floor(2^512 / L)
// (Barrett reduction of a 512-bit value, HAC 14.42 with b = 2^32, k = 8).
ED_CONST uint32_t kL[9] = {0x5CF5D3EDu, 0x5812631Au, 0xA2F79CD6u, 0x14DEF9DEu, 0x00000000u,
                                   0x00000000u, 0x00000000u, 0x10000000u, 0x00000000u};
ED_CONST uint32_t kMu[9] = {0x0A2C131Bu, 0xED9CE5A3u, 0x086329A7u, 0x2106215Du, 0xFFFFFFEBu,
                                    0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x0000000Fu};

// x (16 limbs) mod L into r (8 limbs)
ED_DEV void sc_reduce(const uint32_t (&x)[16], uint32_t (&r)[8]) {
    // q1 = x / b^7 (9 limbs), q2 = q1 mu, q3 = q2 / b^9
    uint32_t q2[18];
    for (int i = 0; i < 18; ++i) q2[i] = 0;
    for (int i = 0; i < 9; ++i) {
        u64 c = 0;
        for (int j = 0; j < 9; ++j) {
            c += (u64)x[7 + i] * kMu[j] + q2[i + j];
            q2[i + j] = (uint32_t)c;
            c >>= 32;
        }
        q2[i + 9] = (uint32_t)c;
    }
    const uint32_t *q3 = q2 + 9;  // 9 limbs
    // r2 = q3 L mod b^9; r = x mod b^9 - r2 (mod b^9)
    uint32_t r2[9];
    for (int i = 0; i < 9; ++i) r2[i] = 0;
    for (int i = 0; i < 9; ++i) {
        u64 c = 0;
        for (int j = 0; i + j < 9; ++j) {
            c += (u64)q3[i] * kL[j] + r2[i + j];
            r2[i + j] = (uint32_t)c;
            c >>= 32;
        }
    }
    uint32_t t[9];
    int64_t s = 0;
    for (int i = 0; i < 9; ++i) {
        s += (int64_t)x[i] - (int64_t)r2[i];
        t[i] = (uint32_t)s;
        s >>= 32;
    }  // (a borrow out of b^9 is the "+ b^(k+1)" of the algorithm: t is that sum)
    for (int k = 0; k < 3; ++k) {  // while t >= L: t -= L
        int ge = 1;
        for (int i = 8; i >= 0; --i) {
            if (t[i] != kL[i]) {
                ge = t[i] > kL[i];
                break;
            }
        }
        if (!ge) break;
        int64_t d = 0;
        for (int i = 0; i < 9; ++i) {
            d += (int64_t)t[i] - (int64_t)kL[i];
            t[i] = (uint32_t)d;
            d >>= 32;
        }
    }
    for (int i = 0; i < 8; ++i) r[i] = t[i];
}

ED_DEV void sc_from_digest(const uint8_t h[64], uint32_t (&r)[8]) {
    uint32_t x[16];
    for (int i = 0; i < 16; ++i)
        x[i] = (uint32_t)h[4 * i] | ((uint32_t)h[4 * i + 1] << 8) | ((uint32_t)h[4 * i + 2] << 16) |
               ((uint32_t)h[4 * i + 3] << 24);
    sc_reduce(x, r);
}

// (a + b c) mod L
ED_DEV void sc_muladd(const uint32_t (&a)[8], const uint32_t (&b)[8], const uint32_t (&c)[8], uint32_t (&r)[8]) {
    uint32_t x[16];
    for (int i = 0; i < 16; ++i) x[i] = i < 8 ? a[i] : 0u;
    for (int i = 0; i < 8; ++i) {
        u64 cy = 0;
        for (int j = 0; j < 8; ++j) {
            cy += (u64)b[i] * c[j] + x[i + j];
            x[i + j] = (uint32_t)cy;
            cy >>= 32;
        }
        for (int k = i + 8; k < 16 && cy; ++k) {
            cy += x[k];
            x[k] = (uint32_t)cy;
            cy >>= 32;
        }
    }
    sc_reduce(x, r);
}

ED_DEV void load_limbs(const uint8_t *b, uint32_t (&r)[8]) {
    for (int i = 0; i < 8; ++i)
        r[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
               ((uint32_t)b[4 * i + 3] << 24);
}

// ------------------------------------------------------------ one item
// PublicKey::verify::<Sha3_512> of ed25519-dalek 0.6: A = 32 bytes (the
// peer's Id), sig = R (32) || S (32), message m of n bytes
ED_DEV bool verify_one(const uint8_t *A, const uint8_t *sig, const uint8_t *m, uint32_t n) {
    const uint8_t *R = sig, *S = sig + 32;
    Pt a;
    if ((S[31] & 224u) != 0 || !pt_decode(A, a)) return false;
    uint8_t h[64];
    sha3_512(Pieces{{R, A, m}, {32u, 32u, n}}, h);
    uint32_t k[8], s[8];
    sc_from_digest(h, k);
    load_limbs(S, s);
    const Pt rp = pt_mul2(s, pt_base(), k, pt_neg(a));  // [S]B - [k]A
    uint8_t enc[32];
    pt_encode(rp, enc);
    uint32_t d = 0;
    for (int b = 0; b < 32; ++b) d |= enc[b] ^ R[b];
    return d == 0;
}

// Keypair::sign::<Sha3_512>: secret seed (32) -> public key A (32) and the
// signature R || S (64) of message m (n bytes)
ED_DEV void sign_one(const uint8_t *seed, const uint8_t *m, uint32_t n, uint8_t *A_out, uint8_t *sig) {
    uint8_t h[64];
    sha3_512(Pieces{{seed, nullptr, nullptr}, {32u, 0u, 0u}}, h);
    h[0] &= 248u;  // clamp: a = 2^254 + 8 * (bits 3..253 of H[0..32])
    h[31] &= 127u;
    h[31] |= 64u;
    uint32_t a[8], zero[8];
    load_limbs(h, a);
    for (int k = 0; k < 8; ++k) zero[k] = 0;
    const Pt B = pt_base();
    uint8_t A[32];
    pt_encode(pt_mul2(a, B, zero, B), A);
    uint8_t hr[64];
    sha3_512(Pieces{{h + 32, m, nullptr}, {32u, n, 0u}}, hr);  // r = H(prefix || M)
    uint32_t r[8];
    sc_from_digest(hr, r);
    uint8_t R[32];
    pt_encode(pt_mul2(r, B, zero, B), R);
    uint8_t hk[64];
    sha3_512(Pieces{{R, A, m}, {32u, 32u, n}}, hk);  // k = H(R || A || M)
    uint32_t k[8], s[8];
    sc_from_digest(hk, k);
    sc_muladd(r, k, a, s);  // S = r + k a mod L
    for (int b = 0; b < 32; ++b) {
        A_out[b] = A[b];
        sig[b] = R[b];
        sig[32 + b] = (uint8_t)(s[b >> 2] >> (8 * (b & 3)));
    }
}

}  // namespace ed
}  // namespace gs
