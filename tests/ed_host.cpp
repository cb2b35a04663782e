// Host build of gs_ed25519.h (test infrastructure): the exact arithmetic the
// GPU kernels of gs_verify.hip run, compiled for the CPU so that
// tests/test_ed25519_host.py can check it against oracle/ed25519_sha3.py
// without a GPU.  Never linked into the product.
#define ED_HOST_TEST
#include "../safe_gossip_amd/csrc/gs_ed25519.h"

extern "C" {
void ed_sha3_512(const uint8_t *m, uint32_t n, uint8_t *out) {
    gs::ed::sha3_512(gs::ed::Pieces{{m, nullptr, nullptr}, {n, 0u, 0u}}, out);
}
int ed_verify(const uint8_t *pub, const uint8_t *sig, const uint8_t *m, uint32_t n) {
    return gs::ed::verify_one(pub, sig, m, n) ? 1 : 0;
}
void ed_sign(const uint8_t *seed, const uint8_t *m, uint32_t n, uint8_t *pub, uint8_t *sig) {
    gs::ed::sign_one(seed, m, n, pub, sig);
}
}
