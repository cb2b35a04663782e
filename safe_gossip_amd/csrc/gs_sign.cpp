// gs_sign.cpp -- host side of the signature half of the wire path
// (gs_verify.hip): batched SHA3-512, ed25519-over-SHA3-512 sign / verify, and
// the signed forms of the engine's byte-level entry points, in which a frame
// is the Message(Vec<u8>, Signature) wrapper of src/messages.rs:26-44.
//
//   Message::serialise   (src/messages.rs:30-34)  -> gs_ed25519_sign, gs_push_batch_signed
//   Message::deserialise (src/messages.rs:36-43)  -> gs_ed25519_verify, gs_handle_received_signed
//
// Keys stay with the caller, as they do with the reference's Gossiper (each
// owns its Keypair, src/gossiper.rs:130-140): a node's 32-byte secret seed is
// passed to the calls that sign for it, and a peer's Id bytes are its public
// key (src/gossiper.rs:84-88).  Every hash and curve operation runs on the
// GPU; the host only packs bytes.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "../../include/safe_gossip.h"
#include "gs_kernels.h"

namespace {

#define GS_HIP(expr)                                   \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) return GS_ERR_HIP;       \
    } while (0)

// Device copies of one batch call, freed on every return path.
struct Batch {
    std::vector<void *> bufs;
    hipStream_t s = nullptr;
    ~Batch() {
        if (s) (void)hipStreamSynchronize(s);
        for (void *p : bufs) (void)hipFree(p);
        if (s) (void)hipStreamDestroy(s);
    }
    template <typename T>
    gs_status put(T **dev, const T *host, size_t count) {
        void *p = nullptr;
        GS_HIP(hipMalloc(&p, count ? count * sizeof(T) : 1));
        bufs.push_back(p);
        if (host && count) GS_HIP(hipMemcpyAsync(p, host, count * sizeof(T), hipMemcpyHostToDevice, s));
        *dev = static_cast<T *>(p);
        return GS_OK;
    }
};

gs_status open_batch(Batch &b, int device) {
    GS_HIP(hipSetDevice(device));
    GS_HIP(hipStreamCreateWithFlags(&b.s, hipStreamNonBlocking));
    return GS_OK;
}

// Total bytes a packed message buffer must hold: max(off[i] + len[i]).
size_t span(uint32_t count, const uint32_t *off, const uint32_t *len) {
    size_t m = 0;
    for (uint32_t i = 0; i < count; ++i) m = std::max(m, (size_t)off[i] + len[i]);
    return m;
}

// Frames "u32 LE length + bytes" of a gs_push_batch / gs_handle_received output.
std::vector<std::pair<uint32_t, uint32_t>> split_frames(const uint8_t *buf, uint32_t len) {
    std::vector<std::pair<uint32_t, uint32_t>> f;
    uint32_t at = 0;
    while (at + 4 <= len) {
        uint32_t n = 0;
        for (int i = 0; i < 4; ++i) n |= (uint32_t)buf[at + i] << (8 * i);
        f.emplace_back(at + 4, n);
        at += 4 + n;
    }
    return f;
}

// Bytes of the signed form of unsigned frames ("u32 length + RPC") totalling
// `unsigned_len` over `count` frames: each becomes "u32 length + Message
// wrapper" (u64 length, RPC, u64 64, 64 signature bytes).
uint32_t signed_size(uint32_t unsigned_len, uint32_t count) { return unsigned_len + count * (8u + 8u + 64u); }

// Replaces every frame of `frames` (RPC bytes) with its signed Message
// wrapper, signed for `seed` on `device`; output frames in `out`.  The size
// is checked before anything is signed (a size query signs nothing).
gs_status sign_frames(int device, const uint8_t seed[32], const std::vector<uint8_t> &frames, uint8_t *out,
                      uint32_t cap, uint32_t *out_len) {
    const auto f = split_frames(frames.data(), (uint32_t)frames.size());
    const uint32_t n = (uint32_t)f.size();
    const uint32_t need = signed_size((uint32_t)frames.size(), n);
    *out_len = need;
    if (!out || cap < need) return GS_ERR_SERIALISATION;
    if (!n) return GS_OK;
    std::vector<uint8_t> seeds(32ull * n);
    std::vector<uint32_t> off(n), len(n);
    for (uint32_t i = 0; i < n; ++i) {
        std::memcpy(&seeds[32ull * i], seed, 32);
        off[i] = f[i].first;
        len[i] = f[i].second;
    }
    std::vector<uint8_t> pub(32ull * n), sig(64ull * n);
    gs_status st = gs_ed25519_sign(device, n, seeds.data(), frames.data(), off.data(), len.data(), pub.data(),
                                   sig.data());
    if (st != GS_OK) return st;
    uint32_t at = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t w = 0;
        const uint32_t m = 8 + len[i] + 8 + 64;
        for (int k = 0; k < 4; ++k) out[at + k] = (uint8_t)(m >> (8 * k));
        st = gs_message_wrap(frames.data() + off[i], len[i], &sig[64ull * i], out + at + 4, m, &w);
        if (st != GS_OK) return st;
        at += 4 + m;
    }
    return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_sha3_512(int device, uint32_t count, const uint8_t *data, const uint32_t *off, const uint32_t *len,
                      uint8_t *out) {
    if (count && (!data || !off || !len || !out)) return GS_ERR_INVALID_ARGUMENT;
    if (!count) return GS_OK;
    Batch b;
    gs_status st = open_batch(b, device);
    const uint8_t *dd = nullptr;
    const uint32_t *doff = nullptr, *dlen = nullptr;
    uint8_t *dout = nullptr;
    if (st == GS_OK) st = b.put(const_cast<uint8_t **>(&dd), data, span(count, off, len));
    if (st == GS_OK) st = b.put(const_cast<uint32_t **>(&doff), off, count);
    if (st == GS_OK) st = b.put(const_cast<uint32_t **>(&dlen), len, count);
    if (st == GS_OK) st = b.put(&dout, (const uint8_t *)nullptr, 64ull * count);
    if (st != GS_OK) return st;
    GS_HIP(gs::launch_sha3_512(dd, doff, dlen, count, dout, b.s));
    GS_HIP(hipMemcpyAsync(out, dout, 64ull * count, hipMemcpyDeviceToHost, b.s));
    GS_HIP(hipStreamSynchronize(b.s));
    return GS_OK;
}

gs_status gs_ed25519_verify(int device, uint32_t count, const uint8_t *pub, const uint8_t *sig, const uint8_t *msg,
                            const uint32_t *off, const uint32_t *len, uint8_t *ok) {
    if (count && (!pub || !sig || !off || !len || !ok || (!msg && span(count, off, len)))) return GS_ERR_INVALID_ARGUMENT;
    if (!count) return GS_OK;
    Batch b;
    gs_status st = open_batch(b, device);
    const uint8_t *dpub = nullptr, *dsig = nullptr, *dmsg = nullptr;
    const uint32_t *doff = nullptr, *dlen = nullptr;
    uint8_t *dok = nullptr;
    if (st == GS_OK) st = b.put(const_cast<uint8_t **>(&dpub), pub, 32ull * count);
    if (st == GS_OK) st = b.put(const_cast<uint8_t **>(&dsig), sig, 64ull * count);
    if (st == GS_OK) st = b.put(const_cast<uint8_t **>(&dmsg), msg, span(count, off, len));
    if (st == GS_OK) st = b.put(const_cast<uint32_t **>(&doff), off, count);
    if (st == GS_OK) st = b.put(const_cast<uint32_t **>(&dlen), len, count);
    if (st == GS_OK) st = b.put(&dok, (const uint8_t *)nullptr, count);
    if (st != GS_OK) return st;
    GS_HIP(gs::launch_ed25519_verify(dpub, dsig, dmsg, doff, dlen, count, dok, b.s));
    GS_HIP(hipMemcpyAsync(ok, dok, count, hipMemcpyDeviceToHost, b.s));
    GS_HIP(hipStreamSynchronize(b.s));
    return GS_OK;
}

gs_status gs_ed25519_sign(int device, uint32_t count, const uint8_t *seed, const uint8_t *msg, const uint32_t *off,
                          const uint32_t *len, uint8_t *pub, uint8_t *sig) {
    if (count && (!seed || !off || !len || !pub || !sig || (!msg && span(count, off, len))))
        return GS_ERR_INVALID_ARGUMENT;
    if (!count) return GS_OK;
    Batch b;
    gs_status st = open_batch(b, device);
    const uint8_t *dseed = nullptr, *dmsg = nullptr;
    const uint32_t *doff = nullptr, *dlen = nullptr;
    uint8_t *dpub = nullptr, *dsig = nullptr;
    if (st == GS_OK) st = b.put(const_cast<uint8_t **>(&dseed), seed, 32ull * count);
    if (st == GS_OK) st = b.put(const_cast<uint8_t **>(&dmsg), msg, span(count, off, len));
    if (st == GS_OK) st = b.put(const_cast<uint32_t **>(&doff), off, count);
    if (st == GS_OK) st = b.put(const_cast<uint32_t **>(&dlen), len, count);
    if (st == GS_OK) st = b.put(&dpub, (const uint8_t *)nullptr, 32ull * count);
    if (st == GS_OK) st = b.put(&dsig, (const uint8_t *)nullptr, 64ull * count);
    if (st != GS_OK) return st;
    GS_HIP(gs::launch_ed25519_sign(dseed, dmsg, doff, dlen, count, dpub, dsig, b.s));
    GS_HIP(hipMemcpyAsync(pub, dpub, 32ull * count, hipMemcpyDeviceToHost, b.s));
    GS_HIP(hipMemcpyAsync(sig, dsig, 64ull * count, hipMemcpyDeviceToHost, b.s));
    GS_HIP(hipStreamSynchronize(b.s));
    return GS_OK;
}

gs_status gs_handle_received_signed(gs_engine *e, uint32_t node, uint32_t peer, const uint8_t peer_key[32],
                                    const uint8_t node_seed[32], const uint8_t *msg, uint32_t msg_len,
                                    uint8_t *out, uint32_t cap, uint32_t *out_len, uint32_t *out_count) {
    if (!e || !peer_key || !msg || !out_len || !out_count) return GS_ERR_INVALID_ARGUMENT;
    *out_len = 0;
    *out_count = 0;
    // Message::deserialise: the wrapper, then the signature over its payload
    uint32_t po = 0, pl = 0, so = 0;
    gs_status st = gs_message_unwrap(msg, msg_len, &po, &pl, &so);
    if (st != GS_OK) return st;
    const uint32_t zero = 0;
    uint8_t ok = 0;
    st = gs_ed25519_verify(gs_device(e), 1, peer_key, msg + so, msg + po, &zero, &pl, &ok);
    if (st != GS_OK) return st;
    if (!ok) return GS_ERR_SIG_FAILURE;  // Error::SigFailure: the frame is dropped, nothing applied
    if (!node_seed) return gs_handle_received(e, node, peer, msg + po, pl, out, cap, out_len, out_count);
    // the Pull responses, signed by the node (Gossiper::prepare_to_send,
    // src/gossiper.rs:117-127).  A size query first: with no room for its
    // responses gs_handle_received applies nothing and reports their unsigned
    // size and count, so the signed size is checked against `cap` before the
    // RPC is applied (nothing applied when it does not fit; call again).  An
    // RPC without responses (a Pull, or a peer already heard from this round)
    // is applied by the query itself, with nothing to sign.
    uint32_t need = 0, cnt = 0;
    st = gs_handle_received(e, node, peer, msg + po, pl, nullptr, 0, &need, &cnt);
    if (st == GS_OK) {
        *out_count = cnt;
        *out_len = need;
        return GS_OK;
    }
    if (st != GS_ERR_SERIALISATION) return st;
    if (!out || cap < signed_size(need, cnt)) {
        *out_len = signed_size(need, cnt);
        return GS_ERR_SERIALISATION;
    }
    std::vector<uint8_t> frames(need);
    uint32_t got = 0;
    st = gs_handle_received(e, node, peer, msg + po, pl, frames.data(), need, &got, &cnt);
    if (st != GS_OK) return st;
    frames.resize(got);
    *out_count = cnt;
    return sign_frames(gs_device(e), node_seed, frames, out, cap, out_len);
}

gs_status gs_push_batch_signed(gs_engine *e, uint32_t node, const uint8_t node_seed[32], uint8_t *out,
                               uint32_t cap, uint32_t *len, uint32_t *count) {
    if (!e || !node_seed || !len || !count) return GS_ERR_INVALID_ARGUMENT;
    uint32_t need = 0;
    gs_status st = gs_push_batch(e, node, nullptr, 0, &need, count);
    if (st != GS_OK && st != GS_ERR_SERIALISATION) return st;
    std::vector<uint8_t> frames(need);
    st = gs_push_batch(e, node, frames.data(), need, &need, count);
    if (st != GS_OK) return st;
    return sign_frames(gs_device(e), node_seed, frames, out, cap, len);
}

}  // extern "C"
