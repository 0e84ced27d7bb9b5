// frame_core.hpp — device-side restatement of nex-packet's Frame semantics
// (shellrow/nex, nex-packet/src/frame.rs:570-658) fused with the packet-API
// verification checksums, written for one lane per frame.
//
// The reference checksums re-serialised packets (ipv4.rs:231-286 to_bytes,
// tcp.rs:521-575, udp.rs:52-60) with a u32 word sum (util.rs:65-183). Here no
// bytes are re-serialised: each checksum is assembled in closed form from
//   * header words read in place, with the fields to_bytes() rewrites
//     substituted (IPv4 IHL/total_length/proto value, TCP data offset, UDP
//     length),
//   * congruent word sums (mod 0xFFFF) of raw byte ranges (`wsum`), and
//   * zero padding where to_bytes() pads.
// A sum T is kept congruent to the reference's u32 sum S modulo 0xFFFF and
// T == 0 iff S == 0 (every weight is positive), which fixes the fold exactly:
// finalize(S) == fold16(T) (util.rs:73-78).
//
// Accessor F (a frame held partly in LDS, partly in HBM) provides:
//   u8(i)      byte i of the frame
//   le_sum(a,b) sum over bytes i in [a,b) of byte * (absolute address of i is
//              odd ? 256 : 1)   (little-endian halfword sum of the range)
// From le_sum the big-endian word sum of [a,b) with words starting at a is
//   a odd  : le_sum(a,b)                 (exactly equal)
//   a even : le_sum(a,b) * 256           (congruent mod 0xFFFF)
// since 65536 == 1 (mod 0xFFFF).  `frame_parity` is the absolute-address
// parity of byte 0, so the parity of byte i is frame_parity ^ (i & 1).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/nexg.h"

// Every function is __host__ __device__: the kernels run it on gfx950 and the
// test-only host harness (tests/native/core_harness.hip) runs the very same
// code on the CPU for differential testing against the oracle.
#define NEXG_HD __host__ __device__ __forceinline__

namespace nexg {

// ip.rs:308-456  IpNextProtocol::new(n).value(): 143..=252 and 255 -> 255.
NEXG_HD uint32_t ip_next_protocol_value(uint32_t n) {
    return (n <= 142u || n == 253u || n == 254u) ? n : 255u;
}

// util.rs:73-78 finalize_checksum on a congruent sum (see header comment).
NEXG_HD uint32_t fold_complement(uint64_t t) {
    t = (t & 0xFFFFFFFFull) + (t >> 32);
    t = (t & 0xFFFFFFFFull) + (t >> 32);
    uint32_t s = (uint32_t)t;
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    return (~s) & 0xFFFFu;
}

// Checksum finisher hook. A plain accessor ignores it; the deferring accessor
// (TileFrame in parse_kernels.hpp) uses it to leave the sum of a long payload
// tail to the cooperative pass and patch the verdict afterwards.
#define NEXG_NO_DEFER                                             \
    NEXG_HD void note_mult(uint32_t) const {}                     \
    NEXG_HD void note_finish(uint64_t, uint32_t, uint32_t) const {}

enum : uint32_t { kCsumIp = 1, kCsumL4 = 2 };

template <class F>
struct FrameOps {
    const F& f;
    uint32_t parity;  // absolute-address parity of frame byte 0

    NEXG_HD uint32_t be16(uint32_t i) const {
        return (f.u8(i) << 8) | f.u8(i + 1);
    }
    NEXG_HD uint32_t be32(uint32_t i) const {
        return (be16(i) << 16) | be16(i + 2);
    }
    // big-endian word sum of [a,b) with words aligned at a (congruent form)
    NEXG_HD uint64_t wsum(uint32_t a, uint32_t b) const {
        if (a >= b) return 0;
        const uint64_t s = f.le_sum(a, b);
        const uint32_t mult = ((parity ^ a) & 1u) ? 1u : 256u;
        f.note_mult(mult);
        return s * mult;
    }
    // fold a finished sum and record the verdict (util.rs:73-78)
    NEXG_HD void finish(uint64_t t, uint32_t stored, uint32_t which, nexg_record& r) const {
        const uint32_t calc = fold_complement(t);
        f.note_finish(t, stored, which);
        if (which == kCsumIp) {
            r.ip_csum_calc = (uint16_t)calc;
            r.flags |= NEXG_C_IP_CHECKED | (calc == stored ? NEXG_C_IP_OK : 0u);
        } else {
            r.l4_csum_calc = (uint16_t)calc;
            r.flags |= NEXG_C_L4_CHECKED | (calc == stored ? NEXG_C_L4_OK : 0u);
        }
    }
};

NEXG_HD void set_payload(nexg_record& r, uint32_t off, uint32_t len) {
    r.payload_off = (uint16_t)(len ? off : 0u);
    r.payload_len = (uint16_t)len;
}

// ---- frame accessors -----------------------------------------------------

// byte mask of dword at slot/abs position j for the byte range [A,B), j < B
NEXG_HD uint32_t range_mask(uint64_t j, uint64_t A, uint64_t B) {
    uint32_t lo = A > j ? (uint32_t)(A - j) : 0u;
    uint32_t hi = (B - j) < 4u ? (uint32_t)(B - j) : 4u;
    uint32_t m = hi >= 4u ? 0xFFFFFFFFu : ((1u << (8u * hi)) - 1u);
    return lo >= 4u ? 0u : (m & (0xFFFFFFFFu << (8u * lo)));
}

NEXG_HD uint32_t halves(uint32_t w) { return (w & 0xFFFFu) + (w >> 16); }

// acc + halves(w) in one instruction on the device (v_sad_u16 against 0)
NEXG_HD uint32_t halves_acc(uint32_t w, uint32_t acc) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sad_u16(w, 0u, acc);
#else
    return acc + halves(w);
#endif
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));

// 16-B global load from a 4-B aligned address (global_load_dwordx4 needs
// dword alignment only); NT = non-temporal
template <bool NT = false>
NEXG_HD uint4 load16a4(const void* p) {
    u32x4a4 v = NT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4a4*>(p))
                   : *reinterpret_cast<const u32x4a4*>(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// Device loads of HBM bytes go through address-space-1 pointers: a
// global_load is counted on vmcnt alone, while a flat load (what a generic
// pointer becomes when the compiler cannot prove it global, e.g. one built
// from an integer address) also counts on lgkmcnt, so the next s_waitcnt
// lgkmcnt(0) for an LDS access, a shuffle or a barrier waits for it too.
#if defined(__HIP_DEVICE_COMPILE__)
#define NEXG_GLOBAL(T, p) reinterpret_cast<const __attribute__((address_space(1))) T*>(reinterpret_cast<uintptr_t>(p))
#else
#define NEXG_GLOBAL(T, p) reinterpret_cast<const T*>(p)
#endif

// 16-B global load; NT = non-temporal (streamed once, do not keep in cache)
template <bool NT = false>
NEXG_HD uint4 load16(const void* p) {
    u32x4 v = NT ? __builtin_nontemporal_load(NEXG_GLOBAL(u32x4, p)) : *NEXG_GLOBAL(u32x4, p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// 16-B global load from an absolute address (k_parse_span's sub-tile
// stream: as a flat load its prefetch was waited for at the next barrier)
template <bool NT = false>
NEXG_HD uint4 load16g(uint64_t addr) {
    return load16<NT>(reinterpret_cast<const void*>(addr));
}

// little-endian halfword sum of global bytes [A, B) (absolute addresses)
NEXG_HD uint64_t global_le_sum(uint64_t A, uint64_t B) {
    uint64_t acc = 0;
    for (uint64_t d = A & ~15ull; d < B; d += 16) {
        const uint4 v = load16(reinterpret_cast<const void*>(d));
        uint32_t s = 0;
        if (d >= A && d + 16 <= B) {
            s = halves(v.x) + halves(v.y) + halves(v.z) + halves(v.w);
        } else {
            if (d + 0 < B) s += halves(v.x & range_mask(d + 0, A, B));
            if (d + 4 < B) s += halves(v.y & range_mask(d + 4, A, B));
            if (d + 8 < B) s += halves(v.z & range_mask(d + 8, A, B));
            if (d + 12 < B) s += halves(v.w & range_mask(d + 12, A, B));
        }
        acc += s;
    }
    return acc;
}

// Frame whose bytes [0, wlen) are staged in an LDS slot (byte i at
// slot[o + i], slot 16-B aligned, o == frame address mod 16) and whose
// remaining bytes are read from HBM.
struct WinFrame {
    NEXG_NO_DEFER
    const uint8_t* slot;
    const uint8_t* g;
    uint32_t o;
    uint32_t wlen;

    NEXG_HD uint32_t u8(uint32_t i) const {
        return i < wlen ? (uint32_t)slot[o + i] : (uint32_t)g[i];
    }
    NEXG_HD uint64_t le_sum(uint32_t a, uint32_t b) const {
        uint64_t acc = 0;
        const uint32_t lb = b < wlen ? b : wlen;
        if (a < lb) {
            const uint32_t A = o + a, B = o + lb;
            const uint32_t* w = reinterpret_cast<const uint32_t*>(slot);
            uint32_t s = 0;
            for (uint32_t j = A & ~3u; j < B; j += 4) s += halves(w[j >> 2] & range_mask(j, A, B));
            acc = s;
        }
        const uint32_t ga = a > wlen ? a : wlen;
        if (ga < b) {
            const uint64_t base = reinterpret_cast<uint64_t>(g);
            acc += global_le_sum(base + ga, base + b);
        }
        return acc;
    }
};

// k_parse_span's generic path: frame bytes [0, 80) in a per-lane LDS slot
// (frame-relative, byte i at slot[i], zero past len), the rest in HBM, and the
// absolute-parity sum of [80, len) already known from the span prefix scan
// (tail; only meaningful when len > 80), or of [80, IP end) for a padded
// frame (span_tail_end). A checksum range that runs to that end (the usual L4
// case) costs no HBM reads past byte 80. Any other
// HBM range longer than kDefer bytes (padded frames: the L4 range ends at the
// IP length) is deferred: le_sum leaves it out and records it, note_mult /
// note_finish record its multiplier and the checksum it feeds, and the caller
// adds the range sum afterwards (the kernel: one wave-wide coalesced pass per
// deferred lane; the host harness: global_le_sum) through span_patch.
struct SpanDeferred {  // 3 dwords: it is live through the whole generic parse
    uint32_t rng = 0;   // frame offset of the range | bytes << 16 (0: nothing deferred)
    uint32_t t = 0;     // the checksum sum without the range, end-around folded
    uint32_t meta = 0;  // stored checksum | which << 16 (0: no checksum took it) | (mult == 256) << 18
    NEXG_HD uint32_t which() const { return (meta >> 16) & 3u; }
    NEXG_HD uint32_t off() const { return rng & 0xFFFFu; }
    NEXG_HD uint32_t bytes() const { return rng >> 16; }
};

// Where k_parse_span takes its second prefix value: the IP end of an
// untagged Ethernet frame whose IPv4 total length / IPv6 payload length ends
// it before the frame end (padding) and at or past byte 84, else the frame
// end. b12 / b16 = little-endian dwords of frame bytes 12..15 / 16..19.
NEXG_HD uint32_t span_tail_end(uint32_t b12, uint32_t b16, uint32_t len, uint32_t opt_flags) {
    if (opt_flags & (NEXG_PARSE_FROM_IP | NEXG_PARSE_VLAN)) return len;
    const uint32_t et = ((b12 & 0xFFu) << 8) | ((b12 >> 8) & 0xFFu);
    const uint32_t e = et == 0x0800u ? 14u + (((b16 & 0xFFu) << 8) | ((b16 >> 8) & 0xFFu))
                     : et == 0x86DDu ? 54u + ((((b16 >> 16) & 0xFFu) << 8) | (b16 >> 24)) : 0u;
    return (e >= 84u && e < len) ? e : len;
}

#ifndef NEXG_SPAN_PROBE
#define NEXG_SPAN_PROBE(k, c)
#endif
#ifndef NEXG_SPAN_SLOT
#define NEXG_SPAN_SLOT 80  // bytes of a declined frame's head in its LDS slot (A/B builds: 128)
#endif
struct SpanFrame {
    static constexpr uint32_t kSlot = NEXG_SPAN_SLOT;
    static_assert(kSlot >= 80 && kSlot % 16 == 0, "the slot holds the 80-B fast-path window");
    static constexpr uint32_t kDefer = 64;
    const uint8_t* slot;
    const uint8_t* g;
    uint32_t tail_end;  // span_tail_end(): the frame end or the IP end of a padded frame
    uint32_t parity;    // absolute-address parity of byte 0
    uint32_t tail;      // absolute-parity sum of [80, tail_end) (when tail_end > 80)
    mutable SpanDeferred d{};
    mutable bool pend = false;

    // one generic (flat) byte load from the slot or HBM: no divergent branch.
    // Only object start + non-negative index here: the compiler keeps one VGPR
    // base per byte run and folds the run's index into the FLAT immediate, and
    // a FLAT access takes its aperture from that VGPR base — a negative
    // displacement of the LDS pointer (round 3's extension windows) put the
    // base below the shared aperture and faulted (profiles/r03/ext_attempt/)
    NEXG_HD uint32_t u8(uint32_t i) const {
        NEXG_SPAN_PROBE(0, i >= kSlot);  // host harness counters (no-op in the library)
        const uint8_t* p = i < kSlot ? slot + i : g + i;
        return *p;
    }
    NEXG_HD uint64_t le_sum(uint32_t a, uint32_t b) const {
        uint64_t acc = 0;
        // a range to tail_end from at most byte 80: [a, 80) from the slot and
        // the scanned tail sum of [80, tail_end); any other range: the slot's
        // part, then HBM past the slot
        const bool to_end = b == tail_end && tail_end > 80u && a <= 80u;
        const uint32_t lb = to_end ? 80u : b < kSlot ? b : kSlot;
        if (a < lb) {  // frame-relative LE sum, x256 for an odd frame (congruent, 0 iff 0)
            const uint32_t* w = reinterpret_cast<const uint32_t*>(slot);
            uint32_t s = 0;
            for (uint32_t j = a & ~3u; j < lb; j += 4) s += halves(w[j >> 2] & range_mask(j, a, lb));
            acc = parity ? (uint64_t)s * 256u : (uint64_t)s;
        }
        const uint32_t ga = a > kSlot ? a : kSlot;
        if (!to_end && ga < b) {
            const uint64_t base = reinterpret_cast<uint64_t>(g);
            if (b - ga > kDefer && d.rng == 0) {
                d.rng = ga | (b - ga) << 16;
                pend = true;
            } else {
                NEXG_SPAN_PROBE(1, true);
                acc += global_le_sum(base + ga, base + b);
            }
        }
        if (to_end) acc += tail;
        return acc;
    }
    NEXG_HD void note_mult(uint32_t m) const {
        if (pend) d.meta = (m == 256u ? 1u : 0u) << 18 | 1u << 20;  // bit 20: multiplier known
        pend = false;
    }
    NEXG_HD void note_finish(uint64_t t, uint32_t stored, uint32_t which) const {
        if ((d.meta >> 20) && !d.which()) {
            t = (t & 0xFFFFFFFFull) + (t >> 32);  // congruent mod 0xFFFF, 0 iff t == 0
            d.t = (uint32_t)((t & 0xFFFFFFFFull) + (t >> 32));
            d.meta = (d.meta & (1u << 18)) | which << 16 | (stored & 0xFFFFu);
        }
    }
};

// finish a deferred checksum: range_sum = le_sum of frame bytes [d.off(), d.off() + d.bytes())
NEXG_HD void span_patch(const SpanDeferred& d, uint64_t range_sum, nexg_record& r) {
    const uint32_t calc = fold_complement((uint64_t)d.t + (((d.meta >> 18) & 1u) ? range_sum * 256u : range_sum));
    const uint32_t stored = d.meta & 0xFFFFu;
    if (d.which() == kCsumIp) {
        r.ip_csum_calc = (uint16_t)calc;
        r.flags = (r.flags & ~NEXG_C_IP_OK) | (calc == stored ? NEXG_C_IP_OK : 0u);
    } else {
        r.l4_csum_calc = (uint16_t)calc;
        r.flags = (r.flags & ~NEXG_C_L4_OK) | (calc == stored ? NEXG_C_L4_OK : 0u);
    }
}

// ---- L4 ------------------------------------------------------------------

// frame.rs:550-568 + udp.rs:197-236 (try_from_bytes) + udp.rs:443-505.
template <class O>
NEXG_HD void parse_udp(const O& o, uint32_t base, uint32_t n,
                                          uint64_t pseudo, nexg_record& r) {
    r.flags |= NEXG_L_TRANSPORT;
    uint32_t ulen = n >= 8 ? o.be16(base + 4) : 0u;
    if (n < 8 || ulen < 8u || n < ulen) {  // Q14
        set_payload(r, base, n);
        return;
    }
    uint32_t sp = o.be16(base), dp = o.be16(base + 2), cs = o.be16(base + 6);
    r.flags |= NEXG_L_UDP;
    r.l4_off = (uint16_t)base;
    r.src_port = (uint16_t)sp;
    r.dst_port = (uint16_t)dp;
    r.l4_length = (uint16_t)ulen;
    r.l4_csum = (uint16_t)cs;
    // to_bytes(): length word rewritten as 8 + payload.len() == ulen; skipword 3
    uint64_t t = pseudo + 17u + ulen + sp + dp + ulen + o.wsum(base + 8, base + ulen);
    o.finish(t, cs, kCsumL4, r);
    set_payload(r, base + 8, ulen - 8);
}

// frame.rs:530-548 + tcp.rs:731-836 (try_from_bytes) + tcp.rs:1207-1269 over
// to_bytes() (tcp.rs:521-575): options re-encoded up to the first EOL, zero
// padded to 4, data offset recomputed; pseudo length = serialised length.
template <class O>
NEXG_HD void parse_tcp(const O& o, uint32_t base, uint32_t n,
                                          uint64_t pseudo, nexg_record& r) {
    r.flags |= NEXG_L_TRANSPORT;
    bool ok = n >= 20;
    uint32_t off_res = ok ? o.f.u8(base + 12) : 0u;
    uint32_t hl = (off_res >> 4) * 4u;
    ok = ok && hl >= 20u && n >= hl;
    uint32_t stop = hl, nopt = 0;
    if (ok) {
        uint32_t off = 20;
        while (off < hl) {
            uint32_t kind = o.f.u8(base + off);
            off += 1;
            if (kind == 0u) {  // EOL: push and stop
                nopt++;
                stop = off;
                break;
            }
            if (kind == 1u) {  // NOP
                nopt++;
                continue;
            }
            if (off >= hl) { ok = false; break; }  // Malformed
            uint32_t l = o.f.u8(base + off);
            off += 1;
            if (l < 2u) { ok = false; break; }  // InvalidLength
            if (off + (l - 2u) > hl) { ok = false; break; }  // Truncated
            nopt++;
            off += l - 2u;
        }
    }
    if (!ok) {  // Q13: transport = Some{None, None}, payload = IP payload
        set_payload(r, base, n);
        return;
    }
    uint32_t sp = o.be16(base), dp = o.be16(base + 2);
    uint32_t seq_hi = o.be16(base + 4), seq_lo = o.be16(base + 6);
    uint32_t ack_hi = o.be16(base + 8), ack_lo = o.be16(base + 10);
    uint32_t flags = o.f.u8(base + 13);
    uint32_t win = o.be16(base + 14), cs = o.be16(base + 16), urg = o.be16(base + 18);
    r.flags |= NEXG_L_TCP;
    r.l4_off = (uint16_t)base;
    r.src_port = (uint16_t)sp;
    r.dst_port = (uint16_t)dp;
    r.tcp_seq = (seq_hi << 16) | seq_lo;
    r.tcp_ack = (ack_hi << 16) | ack_lo;
    r.l4_length = (uint16_t)hl;
    r.l4_type = (uint8_t)flags;
    r.l4_code = (uint8_t)off_res;
    r.tcp_window = (uint16_t)win;
    r.tcp_urg = (uint16_t)urg;
    r.l4_nopt = (uint8_t)nopt;
    r.l4_csum = (uint16_t)cs;
    uint32_t hl_ser = 20u + ((stop - 20u + 3u) & ~3u);
    uint32_t len_ser = hl_ser + (n - hl);
    uint64_t t = pseudo + 6u + len_ser + sp + dp + seq_hi + seq_lo + ack_hi + ack_lo +
                 ((((hl_ser >> 2) << 4) | (off_res & 0xFu)) << 8 | flags) + win + urg +
                 o.wsum(base + 20, base + stop) + o.wsum(base + hl, base + n);
    o.finish(t, cs, kCsumL4, r);
    set_payload(r, base + hl, n - hl);
}

// frame.rs:624-658 + icmp.rs:188-214 / icmpv6.rs:248-272 (>= 8 bytes,
// payload = [4..)); icmp.rs:429 checksum(to_bytes, 1) / icmpv6.rs:589.
template <class O>
NEXG_HD void parse_icmp(const O& o, uint32_t base, uint32_t n,
                                           bool v6, uint64_t pseudo, nexg_record& r) {
    if (n < 8) {  // Q15: icmp = None, payload = IP payload
        set_payload(r, base, n);
        return;
    }
    uint32_t tc = o.be16(base), cs = o.be16(base + 2);
    r.flags |= v6 ? NEXG_L_ICMPV6 : NEXG_L_ICMP;
    r.l4_off = (uint16_t)base;
    r.l4_type = (uint8_t)(tc >> 8);
    r.l4_code = (uint8_t)tc;
    r.l4_csum = (uint16_t)cs;
    uint64_t t = (v6 ? pseudo + 58u + n : 0ull) + tc + o.wsum(base + 4, base + n);
    o.finish(t, cs, kCsumL4, r);
    set_payload(r, base + 4, n - 4);
}

// ---- L3 ------------------------------------------------------------------

// frame.rs:440-483 + ipv4.rs:372-529; ipv4::checksum (ipv4.rs:932-938) over
// to_bytes()[..ihl*4] with the options canonicalised and total_length
// rewritten (Q16/Q17).  Returns the strict-mode ParseError kind or 0.
template <class O>
NEXG_HD uint32_t parse_ipv4(const O& o, uint32_t l3, uint32_t len,
                                               bool strict, nexg_record& r) {
    const uint32_t n = len - l3;
    r.flags |= NEXG_L_IP;
    // err: ParseError kind; ctx / ea / eb: its payload (include/nexg.h NEXG_CTX_*)
    uint32_t err = 0, ctx = 0, ea = 0, eb = 0, hl = 0, total = 0;
    uint32_t b0 = n >= 20u ? o.f.u8(l3) : 0u;
    if (n < 20u) { err = NEXG_ERR_BUFFER_TOO_SHORT; ctx = NEXG_CTX_IPV4_PACKET; ea = 20u; eb = n; }
    else if ((b0 >> 4) != 4u) { err = NEXG_ERR_MALFORMED; ctx = NEXG_CTX_IPV4_VERSION; }
    else if ((b0 & 15u) < 5u) { err = NEXG_ERR_INVALID_LENGTH; ctx = NEXG_CTX_IPV4_HEADER_LENGTH; ea = b0 & 15u; }
    else {
        hl = (b0 & 15u) * 4u;
        if (hl > n) { err = NEXG_ERR_TRUNCATED; ctx = NEXG_CTX_IPV4_HEADER; ea = hl; eb = n; }
        else {
            uint32_t declared = o.be16(l3 + 2);
            uint32_t eff = declared ? declared : n;
            if (eff < hl) { err = NEXG_ERR_INVALID_LENGTH; ctx = NEXG_CTX_IPV4_TOTAL_LENGTH; ea = declared; }
            else if (strict && eff > n) { err = NEXG_ERR_TRUNCATED; ctx = NEXG_CTX_IPV4_PACKET; ea = eff; eb = n; }
            else total = eff < n ? eff : n;
        }
    }
    // options walk (ipv4.rs:442-508): stop = end of the re-serialisable prefix
    uint32_t stop = hl, nopt = 0;
    if (!err) {
        uint32_t i = 20;
        while (i < hl) {
            uint32_t num = o.f.u8(l3 + i) & 0x1Fu;
            if (num == 0u) { nopt++; stop = i + 1; break; }  // EOL
            if (num == 1u) { nopt++; i++; continue; }        // NOP
            if (i + 2u > hl) {
                if (strict) { err = NEXG_ERR_MALFORMED; ctx = NEXG_CTX_IPV4_OPTIONS; }
                stop = i;
                break;
            }
            uint32_t l = o.f.u8(l3 + i + 1);
            if (l < 2u || i + l > hl) {
                if (strict) { err = NEXG_ERR_INVALID_LENGTH; ctx = NEXG_CTX_IPV4_OPTION_LENGTH; ea = l; }
                stop = i;
                break;
            }
            nopt++;
            i += l;
        }
    }
    if (err) {  // Q4: lenient -> ip = Some(all None), payload empty
        if (!strict) return 0u;
        r.l4_type = (uint8_t)ctx;
        r.ip_src = ea;
        r.ip_dst = eb;
        return err;
    }

    uint32_t tos = o.f.u8(l3 + 1);
    uint32_t id = o.be16(l3 + 4), ff = o.be16(l3 + 6);
    uint32_t ttl = o.f.u8(l3 + 8), proto = ip_next_protocol_value(o.f.u8(l3 + 9));
    uint32_t cs = o.be16(l3 + 10);
    uint32_t s_hi = o.be16(l3 + 12), s_lo = o.be16(l3 + 14);
    uint32_t d_hi = o.be16(l3 + 16), d_lo = o.be16(l3 + 18);
    r.flags |= NEXG_L_IPV4;
    r.ip_ver_ihl = (uint8_t)b0;
    r.ip_tos = (uint8_t)tos;
    r.ip_length = (uint16_t)total;
    r.ip_word = (id << 16) | ff;
    r.ip_ttl = (uint8_t)ttl;
    r.ip_proto = (uint8_t)proto;
    r.ip_nopt = (uint8_t)nopt;
    r.ip_src = (s_hi << 16) | s_lo;
    r.ip_dst = (d_hi << 16) | d_lo;
    r.ip_csum = (uint16_t)cs;

    const uint32_t pay = total - hl;
    const uint32_t hl_ser = 20u + ((stop - 20u + 3u) & ~3u);
    if (hl_ser + pay < hl) {
        r.flags |= NEXG_C_IP_PANIC;  // Q17: bytes[..header_len()] out of range
    } else {
        uint32_t tot_ser = hl_ser + pay;
        tot_ser = tot_ser < 65535u ? tot_ser : 65535u;
        uint64_t t = (((0x40u | (hl_ser >> 2)) << 8) | tos) + tot_ser + id + ff +
                     ((ttl << 8) | proto) + s_hi + s_lo + d_hi + d_lo +
                     o.wsum(l3 + 20, l3 + stop) +
                     o.wsum(l3 + hl, l3 + hl + (hl - hl_ser));
        o.finish(t, cs, kCsumIp, r);
    }
    const uint64_t pseudo = (uint64_t)s_hi + s_lo + d_hi + d_lo;  // util.rs:91-93
    const uint32_t pb = l3 + hl;
    if (proto == 6u) parse_tcp(o, pb, pay, pseudo, r);
    else if (proto == 17u) parse_udp(o, pb, pay, pseudo, r);
    else if (proto == 1u) parse_icmp(o, pb, pay, false, pseudo, r);
    else set_payload(r, pb, pay);  // Q9
    return 0;
}

// frame.rs:485-528 + ipv6.rs:217-384. Extension chain walked for the payload
// offset; the Frame dispatches on the raw first next-header (Q10).
template <class O>
NEXG_HD uint32_t parse_ipv6(const O& o, uint32_t l3, uint32_t len,
                                               bool strict, nexg_record& r) {
    const uint32_t n = len - l3;
    r.flags |= NEXG_L_IP;
    // ParseError payload of a strict failure (include/nexg.h NEXG_CTX_*)
    auto fail = [&](uint32_t err, uint32_t ctx, uint32_t ea, uint32_t eb) -> uint32_t {
        if (!strict) return 0u;
        r.l4_type = (uint8_t)ctx;
        r.ip_src = ea;
        r.ip_dst = eb;
        return err;
    };
    if (n < 40u) return fail(NEXG_ERR_BUFFER_TOO_SHORT, NEXG_CTX_IPV6_PACKET, 40u, n);
    uint32_t w0 = o.be32(l3);
    if ((w0 >> 28) != 6u) return fail(NEXG_ERR_MALFORMED, NEXG_CTX_IPV6_VERSION, 0u, 0u);
    uint32_t pl = o.be16(l3 + 4);
    uint32_t declared = 40u + pl;
    if (strict && declared > n) return fail(NEXG_ERR_TRUNCATED, NEXG_CTX_IPV6_PAYLOAD, declared, n);
    uint32_t avail = declared < n ? declared : n;
    uint32_t first = ip_next_protocol_value(o.f.u8(l3 + 6));
    uint32_t nh = first, off = 40, next = 0, ctx = 0, need = 0;
    while (nh == 0u || nh == 43u || nh == 44u || nh == 60u) {
        if (off + 2u > avail) { ctx = NEXG_CTX_IPV6_EXTENSION; need = off + 2u; break; }
        uint32_t nh2 = ip_next_protocol_value(o.f.u8(l3 + off));
        uint32_t el = o.f.u8(l3 + off + 1);
        if (nh == 44u) {
            if (off + 8u > avail) { ctx = NEXG_CTX_IPV6_FRAGMENT; need = off + 8u; break; }
            off += 8u;
        } else {
            if (nh == 43u && off + 4u > avail) { ctx = NEXG_CTX_IPV6_ROUTING; need = off + 4u; break; }
            uint32_t tl = 8u + el * 8u;
            if (off + tl > avail) { ctx = nh == 43u ? NEXG_CTX_IPV6_ROUTING : NEXG_CTX_IPV6_EXTENSION; need = off + tl; break; }
            off += tl;
        }
        next++;
        nh = nh2;
    }
    if (ctx) return fail(NEXG_ERR_TRUNCATED, ctx, need, avail);  // Q12
    r.flags |= NEXG_L_IPV6;
    r.ip_ver_ihl = (uint8_t)((w0 >> 28) << 4);
    r.ip_tos = (uint8_t)(w0 >> 20);
    r.ip_length = (uint16_t)pl;
    r.ip_word = w0 & 0xFFFFFu;
    r.ip_ttl = (uint8_t)o.f.u8(l3 + 7);
    r.ip_proto = (uint8_t)first;
    r.ip_nopt = (uint8_t)(next < 255u ? next : 255u);
    const uint32_t pb = l3 + off, pay = avail - off;
    if (first == 6u || first == 17u || first == 58u) {
        uint64_t pseudo = 0;  // util.rs:135-137 (16 address words)
#pragma unroll
        for (uint32_t k = 0; k < 32; k += 2) pseudo += o.be16(l3 + 8 + k);
        if (first == 6u) parse_tcp(o, pb, pay, pseudo, r);
        else if (first == 17u) parse_udp(o, pb, pay, pseudo, r);
        else parse_icmp(o, pb, pay, true, pseudo, r);
    } else {
        set_payload(r, pb, pay);
    }
    return 0;
}

// frame.rs:424-438 + arp.rs:340-371 (>= 28 bytes; success keeps payload empty)
template <class O>
NEXG_HD void parse_arp(const O& o, uint32_t l3, uint32_t len,
                                          nexg_record& r) {
    const uint32_t n = len - l3;
    if (n < 28u) {
        set_payload(r, l3, n);
        return;
    }
    r.flags |= NEXG_L_ARP;
    r.src_port = (uint16_t)o.be16(l3);
    r.dst_port = (uint16_t)o.be16(l3 + 2);
    r.ip_ver_ihl = (uint8_t)o.f.u8(l3 + 4);
    r.ip_tos = (uint8_t)o.f.u8(l3 + 5);
    r.l4_length = (uint16_t)o.be16(l3 + 6);
    r.ip_src = o.be32(l3 + 14);
    r.ip_dst = o.be32(l3 + 24);
}

// Fast path for the canonical 64-byte Eth/IPv4(IHL 5)/UDP frame (BASELINE
// configs[1] shape) held in registers, w[k] = little-endian dword k of the
// frame. Applies only when the generic path provably yields a plain
// IPv4+UDP Frame whose datagram ends at the frame end: EtherType 0x0800,
// version/IHL 0x45, total_length 50 (or 0 -> captured 50), protocol 17,
// UDP length 30, not FROM_IP. Everything is compile-time indexed; sums use
// BE(word) == 256 * LE(halfword) (mod 0xFFFF). Returns false otherwise (the
// caller runs parse_frame). tests/test_core_harness.py checks both paths.
NEXG_HD bool fast_udp4_64(const uint32_t (&w)[16], uint32_t opt_flags, nexg_record& r) {
    const uint32_t declared = ((w[4] & 0xFFu) << 8) | ((w[4] >> 8) & 0xFFu);
    const uint32_t ulen = (((w[9] >> 16) & 0xFFu) << 8) | (w[9] >> 24);
    const bool ok = (opt_flags & NEXG_PARSE_FROM_IP) == 0u && (w[3] & 0xFFFFFFu) == 0x450008u &&
                    (declared == 50u || declared == 0u) && (w[5] >> 24) == 17u && ulen == 30u;
    if (!ok) return false;
    const uint64_t pseudo = (w[6] >> 16) + halves(w[7]) + (w[8] & 0xFFFFu);
    const uint64_t t_ip = 256ull * ((w[3] >> 16) + (w[4] >> 16) + halves(w[5]) + pseudo) + 50u;
    const uint64_t t_udp = 256ull * (pseudo + (w[8] >> 16) + (w[9] & 0xFFFFu) + (w[10] >> 16) +
                                     halves(w[11]) + halves(w[12]) + halves(w[13]) + halves(w[14]) +
                                     halves(w[15])) + 17u + 30u + 30u;
    const uint32_t ip_calc = fold_complement(t_ip), udp_calc = fold_complement(t_udp);
    const uint32_t ip_cs = ((w[6] & 0xFFu) << 8) | ((w[6] >> 8) & 0xFFu);
    const uint32_t udp_cs = ((w[10] & 0xFFu) << 8) | ((w[10] >> 8) & 0xFFu);
    auto bsw = [](uint32_t x) { return ((x & 0xFFu) << 8) | ((x >> 8) & 0xFFu); };  // BE16 of LE half
    r = nexg_record{};
    r.flags = NEXG_L_ETHERNET | NEXG_L_IP | NEXG_L_IPV4 | NEXG_L_TRANSPORT | NEXG_L_UDP |
              NEXG_C_IP_CHECKED | NEXG_C_L4_CHECKED | (ip_calc == ip_cs ? NEXG_C_IP_OK : 0u) |
              (udp_calc == udp_cs ? NEXG_C_L4_OK : 0u);
    r.payload_off = 42;
    r.payload_len = 22;
    r.packet_len = 64;
    r.ethertype = 0x0800;
    r.l3_off = 14;
    r.l4_off = 34;
    r.ip_ver_ihl = 0x45;
    r.ip_tos = (uint8_t)(w[3] >> 24);
    r.ip_length = 50;
    r.ip_word = (bsw(w[4] >> 16) << 16) | bsw(w[5]);
    r.ip_ttl = (uint8_t)(w[5] >> 16);
    r.ip_proto = 17;
    r.ip_src = (bsw(w[6] >> 16) << 16) | bsw(w[7]);
    r.ip_dst = (bsw(w[7] >> 16) << 16) | bsw(w[8]);
    r.ip_csum = (uint16_t)ip_cs;
    r.ip_csum_calc = (uint16_t)ip_calc;
    r.l4_csum = (uint16_t)udp_cs;
    r.l4_csum_calc = (uint16_t)udp_calc;
    r.src_port = (uint16_t)bsw(w[8] >> 16);
    r.dst_port = (uint16_t)bsw(w[9]);
    r.l4_length = 30;
    return true;
}

// Register fast path over a frame's first 80 bytes: every frame whose Frame
// (frame.rs:570-658) is decided by those bytes plus one L4 tail sum, i.e. the
// canonical IMIX shapes {IPv4 IHL 5, IPv6 without extension headers} x {TCP
// data offset 5, UDP, ICMP/ICMPv6} and the common ways real traffic leaves
// them: TCP option lists of one TLV (NOP, NOP, timestamps / SACK; MSS),
// other EtherTypes (Ethernet only, Q3), an IP header that does not parse (non-strict:
// ip = Some(all None), Q4/Q12), other IP protocols and short
// ICMP (no transport layer, Q9/Q15), a UDP length word that does not fit or a
// TCP header that does not parse (transport layer only, Q14), and IP lengths
// that end the layer before the frame end (Ethernet padding) or past it
// (clamped unless strict). w0[k] holds bytes 4k..4k+3 of the frame
// (little-endian). The window is NOT masked: bytes past `len` (in the span
// kernel the next frame's bytes) reach every read, so no header field may be
// read without an earlier n / data-offset / IP-length check that places it
// before the IP end e (<= len), and the payload sums subtract the window's
// bytes [e, 80) instead of masking them (the host harness poisons the bytes
// past `len` to keep this honest); tail_sum is the frame-relative
// little-endian halfword sum of bytes [80, tail_end) (even frame offsets weigh
// 1, odd 256; 0 when tail_end <= 80) or any value congruent to it mod 0xFFFF
// that is 0 only when it is (callers holding an absolute-parity sum of a frame
// at an odd address pass it x256). The IP layer ends where the reference's
// parse ends it (ipv4.rs:372-529: the declared total length, 0 = the whole
// buffer, clamped to the frame unless strict; ipv6.rs:217-384: 40 + payload
// length, clamped likewise); its checksummed bytes must end at the frame end,
// at tail_end (the span kernel's second prefix value sits there) or inside the
// window (bytes past it masked, no tail). Declined (false, the caller runs
// parse_frame, so the result never depends on which path ran): FROM_IP,
// ARP, VLAN tags under NEXG_PARSE_VLAN, IPv4 options, other TCP options,
// IPv6 extension headers, a UDP datagram shorter than its IP payload,
// strict-mode errors, frames under 14 B. Straight-line selects across the shapes, so a
// mixed wave does not diverge. tests/test_core_harness.py checks it.
NEXG_HD uint32_t wbyte(const uint32_t (&w)[20], uint32_t i) { return (w[i >> 2] >> (8u * (i & 3u))) & 0xFFu; }
NEXG_HD uint32_t wbe16(const uint32_t (&w)[20], uint32_t i) { return (wbyte(w, i) << 8) | wbyte(w, i + 1); }
NEXG_HD uint32_t wle16(const uint32_t (&w)[20], uint32_t i) { return (w[i >> 2] >> (8u * (i & 3u))) & 0xFFFFu; }

NEXG_HD bool fast_canonical80(const uint32_t (&w0)[20], uint32_t len, uint32_t opt_flags,
                              uint64_t tail_sum, uint32_t tail_end, nexg_record& r) {
    if (opt_flags & NEXG_PARSE_FROM_IP) return false;
    if (len < 14u) {  // Q2 (ethernet.rs:310-316), exactly as parse_frame reports it
        r = nexg_record{};
        r.flags = (uint32_t)NEXG_ERR_BUFFER_TOO_SHORT << NEXG_STATUS_SHIFT;
        r.l4_type = NEXG_CTX_ETHERNET_PACKET;
        r.ip_src = 14u;
        r.ip_dst = len;
        return true;
    }
    const uint32_t et = wbe16(w0, 12);
    const bool v6 = et == 0x86DDu, v4 = et == 0x0800u;
    const bool strict = (opt_flags & NEXG_PARSE_STRICT) != 0;
    const uint32_t avail = len - 14u;
    const uint32_t b14 = wbyte(w0, 14), hl = b14 & 15u, decl16 = wbe16(w0, 16);
    // parse_ipv4 / parse_ipv6 failures before the options / extension walk
    const bool bad_ip = v4 ? (avail < 20u || (b14 >> 4) != 4u || hl < 5u || 4u * hl > avail ||
                              (decl16 != 0u && decl16 < 4u * hl))
                           : (avail < 40u || (b14 >> 4) != 6u);
    if (!(v4 || v6) || bad_ip) {
        if ((v4 || v6) ? strict
                       : (et == 0x0806u ||
                          ((opt_flags & NEXG_PARSE_VLAN) && (et == 0x8100u || et == 0x88A8u || et == 0x9100u))))
            return false;
        r = nexg_record{};  // Ethernet only (payload = the rest) or ip = Some(all None) (no payload)
        r.flags = NEXG_L_ETHERNET | ((v4 || v6) ? NEXG_L_IP : 0u);
        r.packet_len = (uint16_t)len;
        r.ethertype = (uint16_t)et;
        r.l3_off = 14;
        if (!(v4 || v6)) {
            r.payload_off = (uint16_t)(avail ? 14u : 0u);
            r.payload_len = (uint16_t)avail;
        }
        return true;
    }
    if (v4 && hl != 5u) return false;  // options
    const uint32_t l4 = v6 ? 54u : 34u;
    const uint32_t decl = v6 ? 40u + wbe16(w0, 18) : (decl16 ? decl16 : avail);
    if (strict && decl > avail) return false;
    const uint32_t ipl = decl < avail ? decl : avail;  // IP bytes parsed (v4: total_length)
    const uint32_t e = 14u + ipl;                      // >= l4
    const uint32_t raw = v6 ? wbyte(w0, 20) : wbyte(w0, 23);
    const uint32_t pv = ip_next_protocol_value(raw);
    if (v6 && (pv == 0u || pv == 43u || pv == 44u || pv == 60u)) {
        // one extension header (hop-by-hop, routing, fragment, destination
        // options) ahead of a non-extension header, inside the IP bytes: the
        // walk of ipv6.rs:217-384 (parse_ipv6) ends after it, and the Frame
        // dispatches on the first next header (Q10): no transport layer and
        // no checksum, the payload follows the extension header
        const uint32_t nh2 = ip_next_protocol_value(wbyte(w0, 54)), el = wbyte(w0, 55);
        const uint32_t tl = pv == 44u ? 8u : 8u + 8u * el;
        if (ipl < 42u || 40u + tl > ipl || nh2 == 0u || nh2 == 43u || nh2 == 44u || nh2 == 60u) return false;
        r = nexg_record{};
        const uint32_t w6 = (wbe16(w0, 14) << 16) | wbe16(w0, 16);
        r.flags = NEXG_L_ETHERNET | NEXG_L_IP | NEXG_L_IPV6;
        r.ip_ver_ihl = 0x60;
        r.ip_tos = (uint8_t)(w6 >> 20);
        r.ip_length = (uint16_t)(decl - 40u);
        r.ip_word = w6 & 0xFFFFFu;
        r.ip_ttl = (uint8_t)wbyte(w0, 21);
        r.ip_proto = (uint8_t)pv;
        r.ip_nopt = 1;
        r.packet_len = (uint16_t)len;
        r.ethertype = (uint16_t)et;
        r.l3_off = 14;
        set_payload(r, 54u + tl, ipl - 40u - tl);
        return true;
    }
    const bool inwin = e <= 80u;  // checksummed bytes all in the window
    if (e != len && e != tail_end && !inwin) return false;
    const uint32_t n = e - l4;
    // the window as given: bytes past e are only ever summed by the payload
    // sums below, which take the bytes [e, 80) back out when e <= 80; every
    // header field read here lies before e whenever it is used
    const uint32_t (&w)[20] = w0;
    if (inwin) tail_sum = 0;
    // the L4 header's dwords, selected once: l4 = 34 / 54 = 2 mod 4, so bytes
    // l4 - 2 .. l4 + 21 are dwords 8..13 / 13..18 and byte l4 + k sits at
    // offset k + 2 of hd (k even: a whole little-endian half of one dword)
    uint32_t hd[6];
#pragma unroll
    for (int j = 0; j < 6; j++) hd[j] = v6 ? w[13 + j] : w[8 + j];
    auto LE = [&](uint32_t k) { return ((k + 2u) & 2u) ? hd[(k + 2u) >> 2] >> 16 : hd[(k + 2u) >> 2] & 0xFFFFu; };
    auto L = [&](uint32_t k) { const uint32_t x = LE(k); return ((x & 0xFFu) << 8) | (x >> 8); };
    const bool tcp = pv == 6u, udp = pv == 17u, icmp = pv == (v6 ? 58u : 1u);
    const uint32_t doff = L(12) >> 12, ulen = L(4);
    const uint32_t o0 = v6 ? w[18] : w[13], o1 = v6 ? w[19] : w[14];
    const uint32_t b20 = (o0 >> 16) & 0xFFu, b21 = o0 >> 24, b22 = o1 & 0xFFu, b23 = (o1 >> 8) & 0xFFu;
    const uint32_t olen = 4u * doff - 20u;  // used when doff > 5
    // an option list whose first option is a TLV with a length below 2 or
    // past the data offset ends the walk of tcp.rs:767-818 with an error
    // (InvalidLength / Truncated): no TcpPacket (Q13), like a short header
    const bool walkfail = doff > 5u && b20 >= 2u && (b21 < 2u || b21 > olen);
    const bool tfail = tcp && (n < 20u || doff < 5u || 4u * doff > n || walkfail);  // no TcpPacket
    const bool q14 = udp && (n < 8u || ulen < 8u || ulen > n);                       // no UdpPacket
    // TCP option lists of one TLV, alone (MSS of a SYN-ACK: 02 04 ..) or
    // behind NOP, NOP (timestamps, RFC 7323's layout for most data segments;
    // SACK blocks), exactly filling the data offset: the option walk
    // (tcp.rs:767-818) gives 1 / 3 options that re-serialise to the same
    // bytes and data offset (tcp.rs:521-575), so the checksum sums the raw
    // bytes from l4 + 20 on like a payload; only the four layout bytes
    // (l4 + 20..23, inside the window for both families) are read
    const bool one = b20 >= 2u && b21 >= 2u && b21 == olen;
    const bool nnx = b20 == 1u && b21 == 1u && b22 >= 2u && b23 >= 2u && 2u + b23 == olen;
    const bool tsopt = tcp && !tfail && doff > 5u && (one || nnx);
    if ((tcp && !tfail && doff != 5u && !tsopt) || (udp && !q14 && ulen != n)) return false;
    const bool tonly = tfail || q14;                                  // transport layer, no packet
    const bool none = !(tcp || udp || icmp) || (icmp && n < 8u);      // no transport layer
    const bool l4ok = !(tonly || none);
    // little-endian suffix sums of the window (bytes >= 4k), for the payload starts
    uint32_t suf[21];
    suf[20] = 0;
#pragma unroll
    for (int k = 19; k >= 0; k--) suf[k] = halves_acc(w[k], suf[k + 1]);
    auto rest = [&](uint32_t s) {  // LE sum of window bytes [s, 80), s even
        return (s & 2u) ? suf[(s >> 2) + 1] + (w[s >> 2] >> 16) : suf[s >> 2];
    };
    const uint32_t h = tcp ? 20u : (udp ? 8u : 4u);
    // s in {38,42,54,58,62,74}: select among compile-time evaluations
    const uint32_t s_start = l4 + h;
    uint32_t rw;
    switch (s_start) {
        case 38: rw = rest(38); break;
        case 42: rw = rest(42); break;
        case 54: rw = rest(54); break;
        case 58: rw = rest(58); break;
        case 62: rw = rest(62); break;
        default: rw = rest(74); break;
    }
    if (inwin) {  // minus the window bytes [e, 80): dword e / 4 from byte e % 4 on, and the dwords after it
        const uint32_t q = e >> 2;
        uint32_t wq = 0, sq = 0;
#pragma unroll
        for (int k = 8; k < 20; k++) {
            const bool m = q == (uint32_t)k;
            wq = m ? w[k] : wq;
            sq = m ? suf[k + 1] : sq;
        }
        rw -= q >= 20u ? 0u : halves_acc(wq & (0xFFFFFFFFu << (8u * (e & 3u))), sq);
    }
    const uint64_t restsum = (uint64_t)rw + tail_sum;
    // pseudo-header address words (LE halves), util.rs:91-93 / 122-123
    // (bytes 22..53 and 26..33 as dword halves: one v_sad_u16 per dword)
    uint32_t p6 = (w[5] >> 16) + (w[13] & 0xFFFFu);
#pragma unroll
    for (int k = 6; k <= 12; k++) p6 = halves_acc(w[k], p6);
    const uint32_t p4 = halves_acc(w[7], (w[6] >> 16) + (w[8] & 0xFFFFu));
    const uint32_t pseudo = v6 ? p6 : p4;
    uint32_t hdr;  // L4 header words other than the checksum (LE halves)
    if (tcp) hdr = halves_acc(hd[3], halves_acc(hd[2], halves_acc(hd[1], (hd[0] >> 16) + (hd[4] & 0xFFFFu) + (hd[5] & 0xFFFFu))));
    else if (udp) hdr = halves_acc(hd[1] & 0xFFFFu, hd[0] >> 16);
    else hdr = hd[0] >> 16;
    uint64_t t4 = 256ull * ((icmp && !v6 ? 0u : pseudo) + hdr + restsum);
    t4 += (icmp && !v6) ? 0u : (pv + n);  // pseudo proto + length (BE constants)
    if (udp) t4 += n;                     // UDP length word as serialised
    const uint32_t l4_calc = fold_complement(t4);
    const uint32_t l4_cs = tcp ? L(16) : (udp ? L(6) : L(2));
    r = nexg_record{};
    uint32_t fl = NEXG_L_ETHERNET | NEXG_L_IP | (v6 ? NEXG_L_IPV6 : NEXG_L_IPV4) | ((tcp || udp) ? NEXG_L_TRANSPORT : 0u);
    if (l4ok)
        fl |= NEXG_C_L4_CHECKED | (l4_calc == l4_cs ? NEXG_C_L4_OK : 0u) |
              (tcp ? NEXG_L_TCP : udp ? NEXG_L_UDP : v6 ? NEXG_L_ICMPV6 : NEXG_L_ICMP);
    if (!v6) {  // ipv4.rs:932-938 over to_bytes(): total_length = 20 + payload, protocol value()
        const uint64_t tip =
            256ull * (wle16(w, 14) + wle16(w, 18) + wle16(w, 20) + (wbyte(w, 22) | pv << 8) + p4) + ipl;
        const uint32_t ip_calc = fold_complement(tip);
        const uint32_t ip_cs = wbe16(w, 24);
        fl |= NEXG_C_IP_CHECKED | (ip_calc == ip_cs ? NEXG_C_IP_OK : 0u);
        r.ip_ver_ihl = 0x45;
        r.ip_tos = (uint8_t)wbyte(w, 15);
        r.ip_length = (uint16_t)ipl;
        r.ip_word = (wbe16(w, 18) << 16) | wbe16(w, 20);
        r.ip_ttl = (uint8_t)wbyte(w, 22);
        r.ip_src = (wbe16(w, 26) << 16) | wbe16(w, 28);
        r.ip_dst = (wbe16(w, 30) << 16) | wbe16(w, 32);
        r.ip_csum = (uint16_t)ip_cs;
        r.ip_csum_calc = (uint16_t)ip_calc;
    } else {
        const uint32_t w6 = (wbe16(w, 14) << 16) | wbe16(w, 16);
        r.ip_ver_ihl = 0x60;
        r.ip_tos = (uint8_t)(w6 >> 20);
        r.ip_length = (uint16_t)(decl - 40u);
        r.ip_word = w6 & 0xFFFFFu;
        r.ip_ttl = (uint8_t)wbyte(w, 21);
    }
    r.flags = fl;
    r.ip_proto = (uint8_t)pv;
    r.packet_len = (uint16_t)len;
    r.ethertype = (uint16_t)et;
    r.l3_off = 14;
    if (!l4ok) {  // frame.rs:530-568 / 624-658: the IP payload is the Frame's payload
        r.payload_off = (uint16_t)(n ? l4 : 0u);
        r.payload_len = (uint16_t)n;
        return true;
    }
    r.l4_off = (uint16_t)l4;
    r.l4_csum = (uint16_t)l4_cs;
    r.l4_csum_calc = (uint16_t)l4_calc;
    if (icmp) {
        r.l4_type = (uint8_t)(L(0) >> 8);
        r.l4_code = (uint8_t)L(0);
    } else {
        r.src_port = (uint16_t)L(0);
        r.dst_port = (uint16_t)L(2);
    }
    if (udp) r.l4_length = (uint16_t)n;
    if (tcp) {
        r.tcp_seq = (L(4) << 16) | L(6);
        r.tcp_ack = (L(8) << 16) | L(10);
        r.l4_length = (uint16_t)(4u * doff);
        r.l4_nopt = tsopt ? (nnx ? 3u : 1u) : 0u;
        r.l4_type = (uint8_t)L(12);
        r.l4_code = (uint8_t)(L(12) >> 8);
        r.tcp_window = (uint16_t)L(14);
        r.tcp_urg = (uint16_t)L(18);
    }
    const uint32_t hp = tsopt ? 4u * doff : h;  // header bytes before the payload
    r.payload_off = (uint16_t)(n > hp ? l4 + hp : 0u);
    r.payload_len = (uint16_t)(n - hp);
    return true;
}

// NEXG_OUT_SPARSE code of a record fast_canonical80 produced, without the
// encoder's shape search: its L4 records are exactly NEXG_SHAPE_V4_UDP ..
// NEXG_SHAPE_V6_ICMP and its records without a transport layer
// NEXG_SHAPE_V4_OTHER / V6_OTHER when the payload runs from the fixed
// headers to the frame end (no VLAN), Ethernet-only and all-None IP records
// are NEXG_SHAPE_ETH_ONLY / IP_NONE; a padded frame or a transport layer
// without a packet (Q14) is an exception (0), as sparse_encode would make it
NEXG_HD uint32_t canonical80_code(const nexg_record& r) {
    const uint32_t f = r.flags;
    if (f >> NEXG_STATUS_SHIFT) return 10u + ((f >> NEXG_STATUS_SHIFT) & 7u);  // BufferTooShort (len < 14): 11
    if (!(f & (NEXG_L_IPV4 | NEXG_L_IPV6))) return (f & NEXG_L_IP) ? (uint32_t)NEXG_SHAPE_IP_NONE : (uint32_t)NEXG_SHAPE_ETH_ONLY;
    const bool v6 = (f & NEXG_L_IPV6) != 0, l4 = (f & NEXG_C_L4_CHECKED) != 0;
    const uint32_t shape = !l4 ? (v6 ? 9u : 8u) : ((v6 ? 4u : 1u) + ((f & NEXG_L_UDP) ? 0u : (f & NEXG_L_TCP) ? 1u : 2u));
    const uint32_t end = !l4 ? (v6 ? 54u : 34u) : r.l4_off + ((f & NEXG_L_UDP) ? 8u : (f & NEXG_L_TCP) ? 20u : 4u);
    const bool coded = (l4 || !(f & NEXG_L_TRANSPORT)) && end + r.payload_len == r.packet_len;
    return coded ? shape | ((f & NEXG_C_IP_OK) ? NEXG_SPARSE_IP_OK : 0u) | ((f & NEXG_C_L4_OK) ? NEXG_SPARSE_L4_OK : 0u)
                 : 0u;
}

// nexg_sparse_decode (include/nexg.h) on the device: the same table macros
NEXG_HD bool sparse_decode(uint32_t code, uint32_t len, uint32_t opt_flags, uint32_t ip_offset, nexg_desc& d) {
    const uint32_t shape = code & 0xFu, tags = (code >> NEXG_SPARSE_TAG_SHIFT) & 3u;
    if (shape == (uint32_t)NEXG_SHAPE_EXCEPTION) return false;
    d.flags = NEXG_SHAPE_FLAGS(shape);
    d.payload_off = 0;
    d.payload_len = 0;
    if (shape >= (uint32_t)NEXG_SHAPE_IP_NONE) {
        if (shape == (uint32_t)NEXG_SHAPE_IP_NONE && tags) d.flags |= NEXG_L_VLAN;
        return true;
    }
    d.flags |= ((code & NEXG_SPARSE_IP_OK) ? NEXG_C_IP_OK : 0u) | ((code & NEXG_SPARSE_L4_OK) ? NEXG_C_L4_OK : 0u) |
               (tags ? NEXG_L_VLAN : 0u);
    const uint32_t h = ((opt_flags & NEXG_PARSE_FROM_IP) ? ip_offset : 14u) + 4u * tags + NEXG_SHAPE_HDR(shape);
    d.payload_len = (uint16_t)(len - h);
    d.payload_off = (uint16_t)(len > h ? h : 0u);
    return true;
}

// NEXG_OUT_SPARSE (include/nexg.h): the 1-B code of a finished record, or 0
// (exception) unless sparse_decode(code, len, ...) reproduces the record's
// descriptor exactly — lossless by construction.
NEXG_HD uint32_t sparse_encode(const nexg_record& r, uint32_t opt_flags, uint32_t ip_offset) {
    const uint32_t st = (r.flags >> NEXG_STATUS_SHIFT) & 7u;
    uint32_t code = 0;
    if (st) {
        code = st == NEXG_ERR_BAD_EXTENT ? 15u : (st <= 4u ? 10u + st : 0u);
    } else {
        const uint32_t base = (opt_flags & NEXG_PARSE_FROM_IP) ? ip_offset : 14u;
        const uint32_t l3 = r.l3_off, tags = (l3 - base) >> 2;
        const uint32_t core = r.flags & ~(NEXG_C_IP_OK | NEXG_C_L4_OK | NEXG_L_VLAN);
        uint32_t shape = 0;
#pragma unroll
        for (uint32_t s = 1; s <= (uint32_t)NEXG_SHAPE_IP_NONE; s++) shape = core == NEXG_SHAPE_FLAGS(s) ? s : shape;
        if (shape == 0u || l3 < base || tags > 2u) return 0u;
        code = shape | ((r.flags & NEXG_C_IP_OK) ? NEXG_SPARSE_IP_OK : 0u) |
               ((r.flags & NEXG_C_L4_OK) ? NEXG_SPARSE_L4_OK : 0u) | (tags << NEXG_SPARSE_TAG_SHIFT);
        const uint32_t hdr = shape < (uint32_t)NEXG_SHAPE_IP_NONE ? NEXG_SHAPE_HDR(shape) : 0u;
        if (base + 4u * tags + hdr > r.packet_len) return 0u;
    }
    nexg_desc d;
    if (!sparse_decode(code, r.packet_len, opt_flags, ip_offset, d)) return 0u;
    return (d.flags == r.flags && d.payload_off == r.payload_off && d.payload_len == r.payload_len) ? code : 0u;
}

// frame.rs:570-607 parse_frame_from_bytes (+ 381-422 dummy Ethernet).
template <class F>
NEXG_HD void parse_frame(const F& f, uint32_t parity, uint32_t len,
                                            uint32_t opt_flags, uint32_t ip_offset,
                                            nexg_record& r) {
    r = nexg_record{};
    FrameOps<F> o{f, parity};
    const bool strict = (opt_flags & NEXG_PARSE_STRICT) != 0u;
    uint32_t ethertype, l3;
    if (opt_flags & NEXG_PARSE_FROM_IP) {
        if (ip_offset >= len) {
            r.flags = (uint32_t)NEXG_ERR_MALFORMED << NEXG_STATUS_SHIFT;
            r.l4_type = NEXG_CTX_DUMMY_ETHERNET;
            return;
        }
        uint32_t n = len - ip_offset, v = f.u8(ip_offset);
        if (n >= 20u && (v >> 4) == 4u && (v & 15u) >= 5u && (v & 15u) * 4u <= n) ethertype = 0x0800u;
        else if (n >= 40u && (v >> 4) == 6u) ethertype = 0x86DDu;
        else {
            r.flags = (uint32_t)NEXG_ERR_MALFORMED << NEXG_STATUS_SHIFT;
            r.l4_type = NEXG_CTX_DUMMY_ETHERNET;
            return;
        }
        l3 = ip_offset;
    } else {
        if (len < 14u) {  // Q2: ethernet.rs:310-316
            r.flags = (uint32_t)NEXG_ERR_BUFFER_TOO_SHORT << NEXG_STATUS_SHIFT;
            r.l4_type = NEXG_CTX_ETHERNET_PACKET;
            r.ip_src = 14u;
            r.ip_dst = len;
            return;
        }
        ethertype = o.be16(12);
        l3 = 14;
    }
    uint32_t vflag = 0;
    if ((opt_flags & (NEXG_PARSE_VLAN | NEXG_PARSE_FROM_IP)) == NEXG_PARSE_VLAN) {
        // extension: up to two tags, each read as vlan.rs:102-127 reads one
        for (int k = 0; k < 2; k++) {
            if (!(ethertype == 0x8100u || ethertype == 0x88A8u || ethertype == 0x9100u) || len < l3 + 4u) break;
            ethertype = o.be16(l3 + 2u);
            l3 += 4u;
            vflag = NEXG_L_VLAN;
        }
    }
    r.packet_len = (uint16_t)len;
    r.ethertype = (uint16_t)ethertype;
    r.l3_off = (uint16_t)l3;
    r.flags = NEXG_L_ETHERNET | vflag;
    uint32_t err = 0;
    if (ethertype == 0x0800u) err = parse_ipv4(o, l3, len, strict, r);
    else if (ethertype == 0x86DDu) err = parse_ipv6(o, l3, len, strict, r);
    else if (ethertype == 0x0806u) parse_arp(o, l3, len, r);
    else set_payload(r, l3, len - l3);  // Q3
    if (err) {  // only the ParseError (kind + payload) survives
        const uint8_t ctx = r.l4_type;
        const uint32_t ea = r.ip_src, eb = r.ip_dst;
        r = nexg_record{};
        r.flags = err << NEXG_STATUS_SHIFT;
        r.l4_type = ctx;
        r.ip_src = ea;
        r.ip_dst = eb;
    }
}

// ---- FrameSlice::try_from_buf (frame.rs:84-287) ---------------------------
// Layer boundaries only (no checksums, no ParseMode): every inner failure is
// an error, AH is walked, ICMP needs 4 B, the UDP length is not checked.

// Field values are kept in locals and the struct is assembled once at the end.
struct SliceAcc {
    uint32_t flags, l3_off, l3_len, l4_len, poff, plen, et;
};

// frame.rs:237-286 parse_transport over [a, a + n); returns a ParseError kind
template <class F>
NEXG_HD uint32_t slice_transport(const F& f, uint32_t proto, uint32_t a, uint32_t n, SliceAcc& s) {
    uint32_t hl = 0;
    if (proto == 6u) {
        if (n >= 20u) {
            hl = (f.u8(a + 12u) >> 4) * 4u;
            if (hl < 20u || hl > n) return NEXG_ERR_INVALID_LENGTH;
        }
    } else if (proto == 17u) {
        hl = n >= 8u ? 8u : 0u;
    } else if (proto == 1u || proto == 58u) {
        hl = n >= 4u ? 4u : 0u;
    }
    if (hl) {
        s.flags |= NEXG_S_TRANSPORT;
        s.l4_len = hl;
    }
    s.poff = a + hl;
    s.plen = n - hl;
    return 0;
}

template <class F>
NEXG_HD uint32_t slice_ip(const F& f, uint32_t et, uint32_t base, uint32_t n, SliceAcc& s) {
    if (et == 0x0800u) {  // frame.rs:138-175
        if (n < 20u) return NEXG_ERR_BUFFER_TOO_SHORT;
        const uint32_t b0 = f.u8(base);
        if ((b0 >> 4) != 4u) return NEXG_ERR_MALFORMED;
        const uint32_t hl = (b0 & 0x0Fu) * 4u;
        if (hl < 20u || hl > n) return NEXG_ERR_INVALID_LENGTH;
        const uint32_t declared = (f.u8(base + 2) << 8) | f.u8(base + 3);
        const uint32_t plen = declared == 0u ? n : (declared < n ? declared : n);
        if (plen < hl) return NEXG_ERR_INVALID_LENGTH;
        const uint32_t proto = ip_next_protocol_value(f.u8(base + 9));
        s.flags |= NEXG_S_NETWORK | NEXG_S_IP_PROTOCOL | (proto << NEXG_S_PROTO_SHIFT);
        s.l3_off = base;
        s.l3_len = hl;
        return slice_transport(f, proto, base + hl, plen - hl, s);
    }
    if (et == 0x86DDu) {  // frame.rs:177-235
        if (n < 40u) return NEXG_ERR_BUFFER_TOO_SHORT;
        if ((f.u8(base) >> 4) != 6u) return NEXG_ERR_MALFORMED;
        const uint32_t declared = (f.u8(base + 4) << 8) | f.u8(base + 5);
        const uint32_t plen = 40u + declared < n ? 40u + declared : n;
        uint32_t next = f.u8(base + 6), cur = 40u;
        while (cur < plen) {
            uint32_t el;
            if (next == 0u || next == 43u || next == 60u) {
                if (cur + 2u > plen) return NEXG_ERR_TRUNCATED;
                el = (f.u8(base + cur + 1) + 1u) * 8u;
            } else if (next == 44u) {
                el = 8u;
            } else if (next == 51u) {
                if (cur + 2u > plen) return NEXG_ERR_TRUNCATED;
                el = (f.u8(base + cur + 1) + 2u) * 4u;
            } else {
                break;
            }
            if (cur + el > plen) return NEXG_ERR_TRUNCATED;
            next = f.u8(base + cur);
            cur += el;
        }
        const uint32_t proto = ip_next_protocol_value(next);
        s.flags |= NEXG_S_NETWORK | NEXG_S_IP_PROTOCOL | (proto << NEXG_S_PROTO_SHIFT);
        s.l3_off = base;
        s.l3_len = cur;
        return slice_transport(f, proto, base + cur, plen - cur, s);
    }
    if (et == 0x0806u && n >= 28u) {  // frame.rs:127-130
        s.flags |= NEXG_S_NETWORK;
        s.l3_off = base;
        s.l3_len = 28u;
        s.poff = base + 28u;
        s.plen = n - 28u;
    }
    return 0;
}

// FrameSlice::try_from_buf (frame.rs:84-136)
template <class F>
NEXG_HD void slice_frame(const F& f, uint32_t len, uint32_t opt_flags, uint32_t ip_offset, nexg_slice& out) {
    SliceAcc s{0, 0, 0, 0, 0, 0, 0};
    uint32_t st = 0;
    if (opt_flags & NEXG_PARSE_FROM_IP) {
        if (ip_offset > len) {
            st = NEXG_ERR_INVALID_LENGTH;
        } else {
            const uint32_t v = ip_offset < len ? (f.u8(ip_offset) >> 4) : 0u;
            if (v == 4u || v == 6u) {
                s.et = v == 4u ? 0x0800u : 0x86DDu;
                s.poff = ip_offset;
                s.plen = len - ip_offset;
            } else {
                st = NEXG_ERR_MALFORMED;
            }
        }
    } else if (len < 14u) {
        st = NEXG_ERR_BUFFER_TOO_SHORT;
    } else {
        s.flags = NEXG_S_DATALINK;
        s.et = (f.u8(12) << 8) | f.u8(13);
        s.poff = 14u;
        s.plen = len - 14u;
    }
    if (st == 0) {
        s.flags |= NEXG_S_ETHERTYPE;
        st = slice_ip(f, s.et, s.poff, s.plen, s);
    }
    out = nexg_slice{};
    if (st) {
        out.flags = st << NEXG_STATUS_SHIFT;
        return;
    }
    out.flags = s.flags;
    out.l3_off = (uint16_t)s.l3_off;
    out.l3_len = (uint16_t)s.l3_len;
    out.l4_len = (uint16_t)s.l4_len;
    out.payload_off = (uint16_t)s.poff;
    out.payload_len = (uint16_t)s.plen;
    out.ethertype = (uint16_t)s.et;
}

}  // namespace nexg
