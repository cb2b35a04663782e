// gs_verify.hip -- the signature half of safe_gossip's wire path on the GPU:
// SHA3-512 (FIPS 202) and ed25519 over SHA3-512, batched one signature per
// lane.
//
//   Message::serialise   (src/messages.rs:30-34): keys.sign::<Sha3_512>(rpc)
//   Message::deserialise (src/messages.rs:36-43): key.verify::<Sha3_512>(msg, sig)
//
// The reference signs through ed25519-dalek ~0.6.1 with the sha3 ~0.7.2
// digest (neither vendored in /root/reference); both are restated here from
// their published algorithms:
//   * SHA3-512: Keccak-f[1600], rate 72 bytes, domain padding 0x06 .. 0x80;
//   * ed25519 (RFC 8032 section 5.1, the hash a parameter): secret expansion
//     a = clamp(H(seed)[0..32]), prefix = H(seed)[32..64]; r = H(prefix || M)
//     mod L, R = [r]B, k = H(R || A || M) mod L, S = r + k a mod L;
//   * verification as ed25519-dalek 0.6 PublicKey::verify: reject when
//     signature[63] & 224 != 0, decompress A (255-bit y reduced mod p), accept
//     iff the encoding of [S]B - [k]A equals the signature's R bytes.
// The CPU restatement oracle/ed25519_sha3.py (pinned by RFC 8032's SHA-512
// vectors) checks these kernels (tests/test_gpu_verify.py); the SHA3-512
// curve results are parity unpinned against a real ed25519-dalek run.
//
// Field elements of GF(2^255 - 19) are 8 little-endian 32-bit limbs holding a
// value below 2^256 (2^256 = 38 mod p folds every carry), reduced to [0, p)
// only to encode or compare.  Points are extended twisted-Edwards coordinates
// (X:Y:Z:T), x = X/Z, y = Y/Z, xy = T/Z, with the unified addition of RFC 8032
// 5.1.4.  Everything is per lane and variable-time (signatures are public);
// throughput is not the point of this path, exactness is.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_ed25519.h"
#include "gs_kernels.h"

namespace gs {
namespace ed {

// ------------------------------------------------------------ kernels
__global__ __launch_bounds__(64) void sha3_batch(const uint8_t *__restrict__ data, const uint32_t *__restrict__ off,
                                                 const uint32_t *__restrict__ len, uint32_t count, uint8_t *out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    Pieces pc = {{data + off[i], nullptr, nullptr}, {len[i], 0u, 0u}};
    uint8_t h[64];
    sha3_512(pc, h);
    for (int k = 0; k < 64; ++k) out[(u64)i * 64 + k] = h[k];
}

// PublicKey::verify::<Sha3_512>(msg, sig) of ed25519-dalek 0.6, one lane each
__global__ __launch_bounds__(64) void verify_batch(const uint8_t *__restrict__ pub, const uint8_t *__restrict__ sig,
                                                   const uint8_t *__restrict__ msg, const uint32_t *__restrict__ off,
                                                   const uint32_t *__restrict__ len, uint32_t count, uint8_t *ok) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    ok[i] = verify_one(pub + 32ull * i, sig + 64ull * i, msg + off[i], len[i]) ? 1u : 0u;
}

// Keypair::sign::<Sha3_512>(msg) for 32-byte secret seeds, one lane each:
// pub[32] and sig[64] out
__global__ __launch_bounds__(64) void sign_batch(const uint8_t *__restrict__ seed, const uint8_t *__restrict__ msg,
                                                 const uint32_t *__restrict__ off, const uint32_t *__restrict__ len,
                                                 uint32_t count, uint8_t *pub, uint8_t *sig) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    sign_one(seed + 32ull * i, msg + off[i], len[i], pub + 32ull * i, sig + 64ull * i);
}

}  // namespace ed

hipError_t launch_sha3_512(const uint8_t *data, const uint32_t *off, const uint32_t *len, uint32_t count,
                           uint8_t *out, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(ed::sha3_batch, dim3((count + 63) / 64), dim3(64), 0, s, data, off, len, count, out);
    return hipGetLastError();
}

hipError_t launch_ed25519_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *msg, const uint32_t *off,
                                 const uint32_t *len, uint32_t count, uint8_t *ok, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(ed::verify_batch, dim3((count + 63) / 64), dim3(64), 0, s, pub, sig, msg, off, len, count, ok);
    return hipGetLastError();
}

hipError_t launch_ed25519_sign(const uint8_t *seed, const uint8_t *msg, const uint32_t *off, const uint32_t *len,
                               uint32_t count, uint8_t *pub, uint8_t *sig, hipStream_t s) {
    if (count == 0) return hipSuccess;
    hipLaunchKernelGGL(ed::sign_batch, dim3((count + 63) / 64), dim3(64), 0, s, seed, msg, off, len, count, pub, sig);
    return hipGetLastError();
}

}  // namespace gs
