// gs_wire.cpp -- the wire format of safe_gossip's RPCs (src/messages.rs):
// bincode (maidsafe_utilities::serialisation, bincode's default fixed-width
// little-endian encoding) of
//   enum GossipRpc { Push { msg: Vec<u8>, counter: u8 }, Pull { .. } }
//   = u32 variant index (0 Push, 1 Pull) | u64 msg length | msg | u8 counter
// and of the signed wrapper Message(Vec<u8>, Signature) used outside
// cfg(test) (src/messages.rs:26-44)
//   = u64 payload length | payload | u64 64 | 64 signature bytes.
// Signing and verification (ed25519 over SHA3-512) are not implemented: no
// library here can check them, so that half is parity-unpinned; frames are
// passed through unverified (the cfg(test) path, src/messages.rs:46-55).
#include <cstring>

#include "../../include/safe_gossip.h"

namespace {

void put_u32(uint8_t *p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
void put_u64(uint8_t *p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
uint32_t get_u32(const uint8_t *p) {
    uint32_t v = 0;
    for (int i = 0; i < 4; ++i) v |= (uint32_t)p[i] << (8 * i);
    return v;
}
uint64_t get_u64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

}  // namespace

extern "C" {

gs_status gs_rpc_encode(int pull, const uint8_t *msg, uint32_t msg_len, uint8_t counter, uint8_t *out,
                        uint32_t cap, uint32_t *out_len) {
    if (!out_len || (msg_len && !msg) || (pull != 0 && pull != 1)) return GS_ERR_INVALID_ARGUMENT;
    const uint64_t need = 4ull + 8ull + msg_len + 1ull;
    *out_len = (uint32_t)need;
    if (need > 0xFFFFFFFFull) return GS_ERR_SERIALISATION;
    if (!out || cap < need) return GS_ERR_SERIALISATION;  // *out_len holds the size needed
    put_u32(out, (uint32_t)pull);
    put_u64(out + 4, msg_len);
    if (msg_len) std::memcpy(out + 12, msg, msg_len);
    out[12 + msg_len] = counter;
    return GS_OK;
}

gs_status gs_rpc_decode(const uint8_t *buf, uint32_t len, int *pull, uint32_t *msg_off, uint32_t *msg_len,
                        uint8_t *counter) {
    if (!buf || !pull || !msg_off || !msg_len || !counter) return GS_ERR_INVALID_ARGUMENT;
    // Message::deserialise (cfg(test)) = maidsafe_utilities::serialisation::
    // deserialise::<GossipRpc> (src/messages.rs:53): an unknown variant or a
    // short buffer is a serialisation error, and so are bytes left over after
    // the RPC (that crate's DeserialiseExtraBytes; recalled, not vendored here)
    if (len < 13) return GS_ERR_SERIALISATION;
    const uint32_t v = get_u32(buf);
    if (v > 1) return GS_ERR_SERIALISATION;
    const uint64_t m = get_u64(buf + 4);
    if (m != (uint64_t)len - 13) return GS_ERR_SERIALISATION;
    *pull = (int)v;
    *msg_off = 12;
    *msg_len = (uint32_t)m;
    *counter = buf[12 + m];
    return GS_OK;
}

gs_status gs_message_wrap(const uint8_t *payload, uint32_t len, const uint8_t signature[64], uint8_t *out,
                          uint32_t cap, uint32_t *out_len) {
    if (!out_len || (len && !payload) || !signature) return GS_ERR_INVALID_ARGUMENT;
    const uint64_t need = 8ull + len + 8ull + 64ull;
    *out_len = (uint32_t)need;
    if (need > 0xFFFFFFFFull) return GS_ERR_SERIALISATION;
    if (!out || cap < need) return GS_ERR_SERIALISATION;
    put_u64(out, len);
    if (len) std::memcpy(out + 8, payload, len);
    put_u64(out + 8 + len, 64);
    std::memcpy(out + 16 + len, signature, 64);
    return GS_OK;
}

gs_status gs_message_unwrap(const uint8_t *buf, uint32_t len, uint32_t *payload_off, uint32_t *payload_len,
                            uint32_t *signature_off) {
    if (!buf || !payload_off || !payload_len || !signature_off) return GS_ERR_INVALID_ARGUMENT;
    // serialisation::deserialise::<Message> (src/messages.rs:37): exactly one
    // wrapper, no bytes after the signature
    if (len < 16) return GS_ERR_SERIALISATION;
    const uint64_t m = get_u64(buf);
    if (m > (uint64_t)len - 16) return GS_ERR_SERIALISATION;
    const uint64_t s = get_u64(buf + 8 + m);
    if (s != 64 || (uint64_t)len != 16 + m + 64) return GS_ERR_SERIALISATION;
    *payload_off = 8;
    *payload_len = (uint32_t)m;
    *signature_off = (uint32_t)(16 + m);
    return GS_OK;
}

}  // extern "C"
