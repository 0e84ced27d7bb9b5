// TEST INFRASTRUCTURE ONLY: runs the engine's device parse core
// (nex_amd/csrc/frame_core.hpp, the exact code the gfx950 kernels execute)
// on the host CPU, reproducing the LaneWindow staging (16-B aligned LDS slot,
// window of `window` bytes, remainder read from "HBM"), so differential tests
// against the oracle run without a GPU. Not part of the product library.
#include <string.h>

// SpanFrame's HBM touches past its LDS bytes, counted by harness_span_groups
static unsigned long long g_span_probe[2];
// byte pattern written past each frame's length where the kernels leave the
// next frame's bytes (harness_set_poison; 0xA5 by default)
static unsigned char g_poison = 0xA5;
extern "C" void harness_set_poison(int v) { g_poison = (unsigned char)v; }
#define NEXG_SPAN_PROBE(k, c) (g_span_probe[k] += (c) ? 1u : 0u)
#include "../../nex_amd/csrc/parse_kernels.hpp"

// tile_of (nexg_internal.hpp, the kernels' workgroup -> tile map) for every
// workgroup of an nb-workgroup grid
extern "C" void harness_tile_map(uint32_t nb, uint32_t order, uint64_t* out) {
    for (uint32_t b = 0; b < nb; b++) out[b] = nexg::tile_of(b, nb, order);
}

extern "C" int harness_parse(const uint8_t* data, uint64_t data_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t stride, uint64_t count,
                             uint32_t flags, uint32_t ip_offset, uint32_t window,
                             int use_fast, nexg_record* out) {
    alignas(16) uint8_t slot[65536 + 32];
    for (uint64_t i = 0; i < count; i++) {
        const uint64_t off = offsets ? offsets[i] : i * (uint64_t)stride;
        const uint64_t len = lengths ? lengths[i] : (offsets ? offsets[i + 1] - off : stride);
        nexg_record r{};
        if (len > 65535 || off > data_bytes || len > data_bytes - off) {
            r.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
        } else {
            const uint8_t* g = data + off;
            const uint32_t o = (uint32_t)(reinterpret_cast<uint64_t>(g) & 15u);
            const uint32_t wlen = len < window ? (uint32_t)len : window;
            memset(slot, g_poison, sizeof(slot));  // poison: bytes outside the window must not matter
            memcpy(slot + o, g, wlen);
            uint32_t w[16];
            if (use_fast && len == 64) memcpy(w, g, 64);
            if (use_fast && len == 64 && nexg::fast_udp4_64(w, flags, r)) {
                out[i] = r;
                continue;
            }
            const uint32_t par = (uint32_t)(reinterpret_cast<uint64_t>(g) & 1u);
            if (use_fast == 4 && (par == 0)) {  // canonical fast path (k_parse_lane80) or generic
                uint32_t w80[20] = {0};
                memcpy(w80, g, len < 80 ? len : 80);
                const uint64_t base = reinterpret_cast<uint64_t>(g);
                const uint64_t tail = len > 80 ? nexg::global_le_sum(base + 80, base + len) : 0;
                if (!nexg::fast_canonical80(w80, (uint32_t)len, flags, tail, (uint32_t)len, r)) {
                    nexg::WinFrame f{slot, g, o, wlen};
                    nexg::parse_frame(f, par, (uint32_t)len, flags, ip_offset, r);
                }
            } else if (use_fast == 5) {
                // k_parse_span's arithmetic at any alignment: the frame re-staged
                // at its own address mod 16 in 16-B chunks; tail sum = Q(end) -
                // Q(80) from running chunk sums + chunk_prefix_sum, in wrapping
                // u32 (absolute parity: x256 for the fast path of an odd frame);
                // declined frames run the generic core on an 80-B slot + that sum
                alignas(16) static uint8_t span[65536 + 64];
                memset(span, 0, sizeof(span));
                memcpy(span + o, g, len);
                auto Q = [&](uint32_t p) {  // prefix at span position p
                    uint32_t q = 0xDEADBEEFu;  // arbitrary running base: only differences matter
                    for (uint32_t c = 0; c < p / 16u; c++) {
                        uint4 v;
                        memcpy(&v, span + 16u * c, 16);
                        q += nexg::chunk_le_sum(v);
                    }
                    const uint32_t m = p & 15u;
                    return q + (m ? nexg::chunk_prefix_sum(span + (p & ~15u), m) : 0u);
                };
                uint32_t w80[20] = {0};
                memcpy(w80, g, len < 80 ? len : 80);
                // the second prefix value at span_tail_end (the IP end of a padded frame)
                const uint32_t te = nexg::span_tail_end(w80[3], w80[4], (uint32_t)len, flags);
                const uint32_t tail = len > 80 ? Q(o + te) - Q(o + 80u) : 0u;
                // the span kernel hands fast_canonical80 its window unmasked: the
                // next frame's bytes past len (here a poison pattern) must not matter
                uint32_t wf[20];
                memset(wf, g_poison, sizeof(wf));
                memcpy(wf, g, len < 80 ? len : 80);
                if (nexg::fast_canonical80(wf, (uint32_t)len, flags, par ? (uint64_t)tail * 256u : tail, te, r)) {
                    // the span kernel stores canonical80_code for these: it must be the encoder's code
                    if (nexg::canonical80_code(r) != nexg::sparse_encode(r, flags, ip_offset)) return -2;
                } else {
                    alignas(16) uint8_t s64[nexg::SpanFrame::kSlot] = {0};  // the slot: head bytes, 0 past len
                    memcpy(s64, g, len < sizeof(s64) ? len : sizeof(s64));
                    nexg::SpanFrame f{s64, g, te, par, tail};
                    nexg::parse_frame(f, par, (uint32_t)len, flags, ip_offset, r);
                    if (f.d.which()) {
                        const uint64_t A = reinterpret_cast<uint64_t>(g) + f.d.off();
                        nexg::span_patch(f.d, nexg::global_le_sum(A, A + f.d.bytes()), r);
                    }
                }
            } else {
                nexg::WinFrame f{slot, g, o, wlen};
                nexg::parse_frame(f, par, (uint32_t)len, flags, ip_offset, r);
            }
        }
        out[i] = r;
    }
    return 0;
}

// FrameSlice core (frame_core.hpp slice_frame) on the host, through the same
// LDS-window accessor the kernels use (window bytes staged, rest "HBM").
extern "C" int harness_slice(const uint8_t* data, uint64_t data_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t stride, uint64_t count,
                             uint32_t flags, uint32_t ip_offset, uint32_t window, nexg_slice* out) {
    alignas(16) uint8_t slot[65536 + 32];
    for (uint64_t i = 0; i < count; i++) {
        const uint64_t off = offsets ? offsets[i] : i * (uint64_t)stride;
        const uint64_t len = lengths ? lengths[i] : (offsets ? offsets[i + 1] - off : stride);
        nexg_slice s{};
        if (len > 65535 || off > data_bytes || len > data_bytes - off) {
            s.flags = (uint32_t)NEXG_ERR_BAD_EXTENT << NEXG_STATUS_SHIFT;
        } else {
            const uint8_t* g = data + off;
            const uint32_t o = (uint32_t)(reinterpret_cast<uint64_t>(g) & 15u);
            const uint32_t wlen = len < window ? (uint32_t)len : window;
            memset(slot, 0xA5, sizeof(slot));
            memcpy(slot + o, g, wlen);
            nexg::WinFrame f{slot, g, o, wlen};
            nexg::slice_frame(f, (uint32_t)len, flags, ip_offset, s);
        }
        out[i] = s;
    }
    return 0;
}

// NEXG_OUT_SPARSE on the host: the kernels' encoder (sparse_encode) over
// records, and both decoders (the kernels' sparse_decode and the C header's
// nexg_sparse_decode) back into descriptors. out_desc[i].flags = 0xFFFFFFFF
// marks an exception code (code 0), which neither decoder resolves.
extern "C" int harness_sparse(const nexg_record* recs, uint64_t count, uint32_t flags, uint32_t ip_offset,
                              uint8_t* codes, nexg_desc* dev_desc, nexg_desc* hdr_desc) {
    for (uint64_t i = 0; i < count; i++) {
        const uint32_t c = nexg::sparse_encode(recs[i], flags, ip_offset);
        codes[i] = (uint8_t)c;
        const uint32_t len = recs[i].packet_len;
        nexg_desc d{0xFFFFFFFFu, 0, 0}, h{0xFFFFFFFFu, 0, 0};
        if (c) {
            if (!nexg::sparse_decode(c, len, flags, ip_offset, d)) return -1;
            if (!nexg_sparse_decode((uint8_t)c, len, flags, ip_offset, &h)) return -1;
        }
        dev_desc[i] = d;
        hdr_desc[i] = h;
    }
    return 0;
}

// both decoders on arbitrary (code, length) pairs; flags 0xFFFFFFFF = exception
extern "C" int harness_sparse_decode(const uint8_t* codes, const uint32_t* lens, uint64_t count, uint32_t flags,
                                     uint32_t ip_offset, nexg_desc* dev_desc, nexg_desc* hdr_desc) {
    for (uint64_t i = 0; i < count; i++) {
        nexg_desc d{0xFFFFFFFFu, 0, 0}, h{0xFFFFFFFFu, 0, 0};
        const bool a = nexg::sparse_decode(codes[i], lens[i], flags, ip_offset, d);
        const bool b = nexg_sparse_decode(codes[i], lens[i], flags, ip_offset, &h) != 0;
        if (a != b) return -1;
        dev_desc[i] = d;
        hdr_desc[i] = h;
    }
    return 0;
}

// k_parse_span's generic section for packed batches, group by group, on the
// host: the workgroup's LDS slots emulated by one 20480-B heap block (so an
// AddressSanitizer build catches any slot access outside it), the fast path on
// every frame's head window with the scanned tail sum, declined frames
// bucketed in lane order, the generic core on SpanFrame, deferred ranges
// patched; harness_span_stats counts what the generic section does.
// Records out (the record form of what the sparse kernel encodes). Frames of a
// group that is not packed (or a batch that is not) return -1.
static uint8_t* g_span_declined;  // optional per-frame output: 1 = the generic core parsed it
extern "C" void harness_span_declined(uint8_t* out) { g_span_declined = out; }
static uint64_t g_span_stats[6];  // declined, declined past 80 B, deferred ranges, groups with a declined
                                  // frame, HBM byte loads, inline HBM range sums (the last two: NEXG_SPAN_PROBE)
extern "C" const uint64_t* harness_span_stats() {
    g_span_stats[4] = g_span_probe[0];
    g_span_stats[5] = g_span_probe[1];
    return g_span_stats;
}
extern "C" void harness_span_stats_reset() {
    for (auto& v : g_span_stats) v = 0;
    g_span_probe[0] = g_span_probe[1] = 0;
}
extern "C" int harness_span_groups(const uint8_t* data, uint64_t data_bytes, const uint64_t* offsets,
                                   uint64_t count, uint32_t flags, uint32_t ip_offset, nexg_record* out) {
    constexpr uint32_t T = nexg::kTile, S = nexg::SpanFrame::kSlot, W = nexg::kLaneWin;
    uint8_t* lds = static_cast<uint8_t*>(aligned_alloc(16, T * S));
    const uint64_t base = reinterpret_cast<uint64_t>(data);
    for (uint64_t f0 = 0; f0 < count; f0 += T) {
        const uint32_t nf = count - f0 < T ? (uint32_t)(count - f0) : T;
        const uint64_t lo = offsets[f0], hi = offsets[f0 + nf];
        if (hi < lo || hi > data_bytes) { free(lds); return -1; }
        const uint64_t A0 = (base + lo) & ~15ull;
        memset(lds, 0xA5, T * S);
        bool gen[T] = {};
        uint32_t key[T] = {}, hr[T] = {}, len[T] = {}, qend[T] = {}, tq[T] = {};
        for (uint32_t t = 0; t < nf; t++) {
            const uint64_t off = offsets[f0 + t], l = offsets[f0 + t + 1] - off;
            if (l > 65535 || off < lo || off + l > hi) { free(lds); return -1; }
            len[t] = (uint32_t)l;
            hr[t] = (uint32_t)(base + off - A0);
            const uint8_t* g = data + off;
            uint32_t w[S / 4] = {0};  // the slot's bytes (the first W: the fast path's window)
            memcpy(w, g, l < S ? l : S);
            uint32_t wf[20];  // as the kernel: the window unmasked past len (the batch's next bytes)
            memset(wf, 0x5A, sizeof(wf));
            memcpy(wf, g, (uint64_t)W <= (uint64_t)(data + data_bytes - g) ? W : (size_t)(data + data_bytes - g));
            qend[t] = nexg::span_tail_end(w[3], w[4], len[t], flags);
            uint32_t q = 0;  // absolute-parity LE sum of [80, qend): Q(end) - Q(start + 80)
            for (uint32_t k = W; k < qend[t]; k++) q += (uint32_t)g[k] << (((base + off + k) & 1u) ? 8u : 0u);
            tq[t] = len[t] > W ? q : 0u;
            nexg_record r{};
            const uint64_t tail = ((base + off) & 1u) ? (uint64_t)tq[t] * 256u : (uint64_t)tq[t];
            if (nexg::fast_canonical80(wf, len[t], flags, tail, qend[t], r)) {
                out[f0 + t] = r;
            } else {
                gen[t] = true;
                if (g_span_declined) g_span_declined[f0 + t] = 1;
                key[t] = nexg::span_bucket(w[3], w[5], flags);
                memcpy(lds + S * t, w, S);
            }
        }
        // items in bucket order (lane order inside a bucket)
        uint32_t ngen = 0, items[T];
        for (uint32_t b = 0; b < nexg::kBuckets; b++)
            for (uint32_t t = 0; t < nf; t++)
                if (gen[t] && key[t] == b) items[ngen++] = t;
        g_span_stats[3] += ngen > 0;
        for (uint32_t ii = 0; ii < ngen; ii++) {
            const uint32_t t = items[ii];
            nexg_record rr{};
            nexg::SpanFrame f{lds + S * t, reinterpret_cast<const uint8_t*>(A0 + hr[t]), qend[t], hr[t] & 1u, tq[t]};
            nexg::parse_frame(f, hr[t] & 1u, len[t], flags, ip_offset, rr);
            g_span_stats[0]++;
            g_span_stats[1] += len[t] > W;
            g_span_stats[2] += f.d.which() != 0;
            if (f.d.which()) {
                const uint64_t A = A0 + hr[t] + f.d.off();
                nexg::span_patch(f.d, nexg::global_le_sum(A, A + f.d.bytes()), rr);
            }
            out[f0 + t] = rr;
        }
    }
    free(lds);
    return 0;
}
