// nexg_api.hip — the C ABI declared in include/nexg.h.
//
// Validation, context handling and kernel selection only; every byte of frame
// data is processed by the gfx950 kernels in nexg_parse.hip / nexg_build.hip.
// There is deliberately no CPU fallback: a missing or non-gfx950 device makes
// nexg_ctx_create fail with NEXG_EDEVICE.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nexg_internal.hpp"

struct nexg_ctx {
    int device;
    int cu_count;
    char arch[64];
    char last_error[256];
    void* scratch;          // device memory for per-call hand-offs (TwoPass tail sums)
    uint64_t scratch_bytes;
    hipEvent_t scratch_done;    // recorded after the last launch that used the scratch ...
    hipStream_t scratch_stream; // ... on this stream
    bool scratch_used;
};

namespace {

// Every entry point runs with the context's device current and restores the
// caller's afterwards: allocations and NULL-stream launches then land on the
// device the context is bound to, whichever device the thread had selected.
struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    explicit DeviceGuard(const nexg_ctx* ctx) {
        if (ctx && hipGetDevice(&prev) == hipSuccess && prev != ctx->device)
            switched = hipSetDevice(ctx->device) == hipSuccess;
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
};

// ctx scratch of at least `bytes` (grown, never shrunk; hipFree is
// device-synchronous, so no launch still reads the old block)
void* scratch(nexg_ctx* ctx, uint64_t bytes) {
    if (ctx->scratch_bytes >= bytes) return ctx->scratch;
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    ctx->scratch = nullptr;
    ctx->scratch_bytes = 0;
    const uint64_t want = bytes < (1ull << 20) ? (1ull << 20) : bytes;
    if (hipMalloc(&ctx->scratch, want) != hipSuccess) {
        ctx->scratch = nullptr;
        return nullptr;
    }
    ctx->scratch_bytes = want;
    return ctx->scratch;
}

// The scratch is shared by every call on the context, whatever its stream:
// a call on another stream than the last user's waits for that user's launch
// (stream order alone covers calls on one stream).
hipError_t scratch_acquire(nexg_ctx* ctx, hipStream_t stream) {
    if (!ctx->scratch_used || ctx->scratch_stream == stream) return hipSuccess;
    return hipStreamWaitEvent(stream, ctx->scratch_done, 0);
}

hipError_t scratch_release(nexg_ctx* ctx, hipStream_t stream) {
    if (!ctx->scratch_done) {
        const hipError_t e = hipEventCreateWithFlags(&ctx->scratch_done, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    const hipError_t e = hipEventRecord(ctx->scratch_done, stream);
    if (e != hipSuccess) return e;
    ctx->scratch_stream = stream;
    ctx->scratch_used = true;
    return hipSuccess;
}

int fail(nexg_ctx* ctx, int code, const char* fmt, const char* detail) {
    if (ctx) snprintf(ctx->last_error, sizeof(ctx->last_error), fmt, detail ? detail : "");
    return code;
}

int hip_status(nexg_ctx* ctx, hipError_t e, int code) {
    if (e == hipSuccess) return NEXG_OK;
    return fail(ctx, code, "HIP: %s", hipGetErrorString(e));
}

bool frames_valid(const nexg_frames* f) {
    if (!f) return false;
    if (f->count == 0) return true;
    if (!f->data) return false;
    if (!f->offsets && f->stride == 0) return false;
    if ((reinterpret_cast<uint64_t>(f->data) & 3u) != 0) return false;  // 4-B aligned base
    if ((f->hints & NEXG_FRAMES_OFFSETS32) && (reinterpret_cast<uint64_t>(f->offsets) & 3u) != 0) return false;
    return true;
}

nexg::ParseArgs to_args(const nexg_frames* f) {
    nexg::ParseArgs a{};
    a.data = f->data;
    a.data_bytes = f->data_bytes;
    a.offsets = f->offsets;
    a.lengths = f->lengths;
    a.stride = f->stride;
    a.count = f->count;
    a.hints = f->hints;
    if ((f->hints & NEXG_FRAMES_OFFSETS32) && f->offsets && f->data_bytes > 0xFFFFFFFFull)
        a.off_bases = nexg_offsets32_bases(f->offsets, f->count);
    return a;
}

}  // namespace

extern "C" {

int nexg_abi_version(void) { return NEXG_ABI_VERSION; }

const char* nexg_strerror(int status) {
    switch (status) {
        case NEXG_OK: return "ok";
        case NEXG_EINVAL: return "invalid argument";
        case NEXG_ENOMEM: return "out of memory";
        case NEXG_EDEVICE: return "device error or device is not gfx950";
        case NEXG_ELAUNCH: return "kernel launch failed";
        case NEXG_ERANGE: return "length overflow (BuildError::LengthOverflow)";
        default: return "unknown status";
    }
}

int nexg_ctx_create(int device, nexg_ctx** out) {
    if (!out) return NEXG_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return NEXG_EDEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return NEXG_EDEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return NEXG_EDEVICE;
    nexg_ctx* c = static_cast<nexg_ctx*>(calloc(1, sizeof(nexg_ctx)));
    if (!c) return NEXG_ENOMEM;
    c->device = device;
    c->cu_count = prop.multiProcessorCount;
    snprintf(c->arch, sizeof(c->arch), "%s", prop.gcnArchName);
    *out = c;
    return NEXG_OK;
}

int nexg_ctx_destroy(nexg_ctx* ctx) {
    if (ctx && (ctx->scratch || ctx->scratch_done)) {
        DeviceGuard g(ctx);
        if (ctx->scratch) (void)hipFree(ctx->scratch);
        if (ctx->scratch_done) (void)hipEventDestroy(ctx->scratch_done);
    }
    free(ctx);
    return NEXG_OK;
}

const char* nexg_ctx_last_error(const nexg_ctx* ctx) { return ctx ? ctx->last_error : ""; }

int nexg_ctx_cu_count(const nexg_ctx* ctx) { return ctx ? ctx->cu_count : 0; }

int nexg_parse_batch(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                     int out_kind, void* out, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!frames_valid(frames)) return fail(ctx, NEXG_EINVAL, "invalid frame batch%s", nullptr);
    if (out_kind != NEXG_OUT_DESC && out_kind != NEXG_OUT_RECORD && out_kind != NEXG_OUT_SLICE &&
        out_kind != NEXG_OUT_FLAGS && out_kind != NEXG_OUT_VERDICT && out_kind != NEXG_OUT_SPARSE &&
        out_kind != NEXG_OUT_GROUPED)
        return fail(ctx, NEXG_EINVAL, "invalid out_kind%s", nullptr);
    if (frames->count && !out) return fail(ctx, NEXG_EINVAL, "NULL output%s", nullptr);
    const uint64_t align_mask = out_kind == NEXG_OUT_VERDICT ? 1u : out_kind == NEXG_OUT_FLAGS ? 3u
                                : out_kind == NEXG_OUT_DESC  ? 7u : 15u;
    if ((reinterpret_cast<uint64_t>(out) & align_mask) != 0)
        return fail(ctx, NEXG_EINVAL, "misaligned output%s", nullptr);
    DeviceGuard g(ctx);
    nexg::ParseArgs a = to_args(frames);
    a.opt_flags = option ? option->flags : 0u;
    a.ip_offset = option ? option->ip_offset : 0u;
    a.out = out;
    a.tile_order = nexg::tile_order_for(a);
    const nexg::ParseVariant v = nexg::choose_parse_variant(a);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    if (nexg::parse_needs_tail(v, out_kind) && a.count) {
        a.tail = static_cast<uint32_t*>(scratch(ctx, a.count * 4u));
        if (!a.tail) return fail(ctx, NEXG_ENOMEM, "device scratch allocation failed%s", nullptr);
        if (int rc = hip_status(ctx, scratch_acquire(ctx, st), NEXG_ELAUNCH)) return rc;
        if (int rc = hip_status(ctx, nexg::launch_parse(v, a, out_kind, st), NEXG_ELAUNCH)) return rc;
        return hip_status(ctx, scratch_release(ctx, st), NEXG_ELAUNCH);
    }
    return hip_status(ctx, nexg::launch_parse(v, a, out_kind, st), NEXG_ELAUNCH);
}

static int sparse_expand(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                         const void* sparse, nexg_desc* out, bool grouped, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!frames_valid(frames)) return fail(ctx, NEXG_EINVAL, "invalid frame batch%s", nullptr);
    if (frames->count && (!sparse || !out)) return fail(ctx, NEXG_EINVAL, "NULL sparse input or output%s", nullptr);
    if (((reinterpret_cast<uint64_t>(sparse) & 15u) | (reinterpret_cast<uint64_t>(out) & 7u)) != 0)
        return fail(ctx, NEXG_EINVAL, "misaligned sparse input or output%s", nullptr);
    DeviceGuard g(ctx);
    nexg::ParseArgs a = to_args(frames);
    a.opt_flags = option ? option->flags : 0u;
    a.ip_offset = option ? option->ip_offset : 0u;
    return hip_status(ctx, nexg::launch_sparse_expand(a, static_cast<const uint8_t*>(sparse), out, grouped,
                                                      static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_sparse_expand(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                       const void* sparse, nexg_desc* out, void* stream) {
    return sparse_expand(ctx, frames, option, sparse, out, false, stream);
}

int nexg_grouped_expand(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                        const void* grouped, nexg_desc* out, void* stream) {
    return sparse_expand(ctx, frames, option, grouped, out, true, stream);
}

int nexg_recompute_checksums_batch(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option,
                                   uint32_t which, nexg_fixup* out, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!frames_valid(frames)) return fail(ctx, NEXG_EINVAL, "invalid frame batch%s", nullptr);
    if ((which & ~(NEXG_FIX_IP | NEXG_FIX_L4)) != 0) return fail(ctx, NEXG_EINVAL, "invalid fix-up selection%s", nullptr);
    if ((reinterpret_cast<uint64_t>(out) & 7u) != 0) return fail(ctx, NEXG_EINVAL, "misaligned output%s", nullptr);
    DeviceGuard g(ctx);
    nexg::ParseArgs a = to_args(frames);
    a.opt_flags = option ? option->flags : 0u;
    a.ip_offset = option ? option->ip_offset : 0u;
    return hip_status(ctx, nexg::launch_recompute(a, which, out, static_cast<hipStream_t>(stream)), NEXG_ELAUNCH);
}

int nexg_checksum_batch(nexg_ctx* ctx, const nexg_frames* bufs, uint32_t skipword, uint16_t* out,
                        void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!frames_valid(bufs)) return fail(ctx, NEXG_EINVAL, "invalid buffer batch%s", nullptr);
    if (bufs->count && !out) return fail(ctx, NEXG_EINVAL, "NULL output%s", nullptr);
    nexg::ParseArgs a = to_args(bufs);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_checksum(a, skipword, out, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_decode_options(nexg_ctx* ctx, const nexg_frames* frames, const nexg_record* records,
                        nexg_options* out, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!frames_valid(frames)) return fail(ctx, NEXG_EINVAL, "invalid frame batch%s", nullptr);
    if (frames->count && (!records || !out)) return fail(ctx, NEXG_EINVAL, "NULL records or output%s", nullptr);
    if ((reinterpret_cast<uint64_t>(out) & 15u) != 0 || (reinterpret_cast<uint64_t>(records) & 15u) != 0)
        return fail(ctx, NEXG_EINVAL, "misaligned records or output%s", nullptr);
    const nexg::ParseArgs a = to_args(frames);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_decode_options(a, records, out, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_probe_stream(nexg_ctx* ctx, const void* data, uint64_t bytes, uint32_t out_per_64,
                      void* out, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    const bool wo = out_per_64 == 64;  // write-only: data unused
    if (bytes % 16384u != 0 || (bytes && ((!wo && !data) || !out)) ||
        (out_per_64 != 0 && out_per_64 != 8 && out_per_64 != 9 && !wo) || (reinterpret_cast<uint64_t>(data) & 15u) != 0 ||
        (reinterpret_cast<uint64_t>(out) & (wo ? 15u : 7u)) != 0)
        return fail(ctx, NEXG_EINVAL, "probe: bytes must be a multiple of 16384, buffers aligned%s", nullptr);
    if (bytes / 16384u > 0x7FFFFFFFull) return fail(ctx, NEXG_ERANGE, "probe: too many tiles%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_probe_stream(static_cast<const uint8_t*>(data), bytes / 16384u,
                                                     out_per_64, out, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_probe_span_clock(nexg_ctx* ctx, const nexg_frames* frames, const nexg_parse_option* option, void* out,
                          uint64_t* stamps, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!frames_valid(frames)) return fail(ctx, NEXG_EINVAL, "invalid frame batch%s", nullptr);
    if (frames->count && (!out || !stamps)) return fail(ctx, NEXG_EINVAL, "NULL output or stamps%s", nullptr);
    if (((reinterpret_cast<uint64_t>(out) & 15u) | (reinterpret_cast<uint64_t>(stamps) & 7u)) != 0)
        return fail(ctx, NEXG_EINVAL, "misaligned output or stamps%s", nullptr);
    DeviceGuard g(ctx);
    nexg::ParseArgs a = to_args(frames);
    a.opt_flags = option ? option->flags : 0u;
    a.ip_offset = option ? option->ip_offset : 0u;
    a.out = out;
    a.tile_order = nexg::tile_order_for(a);
    a.stamps = stamps;
    if (nexg::choose_parse_variant(a) != nexg::ParseVariant::SpanTile)
        return fail(ctx, NEXG_EINVAL, "probe_span_clock: the batch does not take the span kernel%s", nullptr);
    return hip_status(ctx, nexg::launch_span_clock(a, static_cast<hipStream_t>(stream)), NEXG_ELAUNCH);
}

int nexg_probe_latency(nexg_ctx* ctx, void* buf, uint64_t bytes, uint32_t steps, uint32_t start, uint32_t loaded,
                       uint64_t* out, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (!buf || !out || bytes < 64u * 65536u || bytes / 64u > 0xFFFFFFFFull || steps == 0 || steps > (1u << 20) ||
        (reinterpret_cast<uint64_t>(buf) & 15u) != 0 || (reinterpret_cast<uint64_t>(out) & 7u) != 0)
        return fail(ctx, NEXG_EINVAL, "probe_latency: buffer of at least 4 MiB (16-B aligned), 1..2^20 steps%s", nullptr);
    DeviceGuard g(ctx);
    // loaded: one reading workgroup per CU x 4, at most 64 passes over the buffer
    const uint32_t wgs = loaded ? (uint32_t)ctx->cu_count * 4u : 0u;
    return hip_status(ctx, nexg::launch_probe_latency(static_cast<uint32_t*>(buf), (uint32_t)(bytes / 64u), start, steps,
                                                      wgs, 64u, out, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_build_udp4_batch(nexg_ctx* ctx, const nexg_udp4_build* p, uint8_t* out,
                          uint32_t out_stride, void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (28ull + p->payload_len > 65535ull)
        return fail(ctx, NEXG_ERANGE, "UDP/IPv4 length overflow%s", nullptr);
    if (p->count && (!p->dst_ip || !out))
        return fail(ctx, NEXG_EINVAL, "NULL address array or output%s", nullptr);
    if (p->payload_len && !p->payload) return fail(ctx, NEXG_EINVAL, "NULL payload%s", nullptr);
    if (out_stride < 42u + p->payload_len)
        return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_udp4(*p, out, out_stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_build_udp4_tuples(nexg_ctx* ctx, const nexg_udp4_build* p, const nexg_udp4_tuple* tuples, uint8_t* out,
                           uint32_t out_stride, void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (28ull + p->payload_len > 65535ull)
        return fail(ctx, NEXG_ERANGE, "UDP/IPv4 length overflow%s", nullptr);
    if (p->src_ip || p->dst_ip || p->src_port || p->dst_port || p->ip_id || p->src_mac || p->dst_mac)
        return fail(ctx, NEXG_EINVAL, "per-frame arrays come from the tuples: pass NULL%s", nullptr);
    if (p->count && (!tuples || !out))
        return fail(ctx, NEXG_EINVAL, "NULL tuples or output%s", nullptr);
    if ((reinterpret_cast<uint64_t>(tuples) & 15u) != 0)
        return fail(ctx, NEXG_EINVAL, "tuples must be 16-B aligned%s", nullptr);
    if (p->payload_len && !p->payload) return fail(ctx, NEXG_EINVAL, "NULL payload%s", nullptr);
    if (out_stride < 42u + p->payload_len)
        return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_udp4_tuples(*p, tuples, out, out_stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_build_udp6_batch(nexg_ctx* ctx, const nexg_udp6_build* p, uint8_t* out,
                          uint32_t out_stride, void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (8ull + p->payload_len > 65535ull)
        return fail(ctx, NEXG_ERANGE, "UDP/IPv6 length overflow%s", nullptr);
    // src_ip is per frame here (no def_src_ip: only the IPv4 probe batch has one)
    if (p->count && (!p->src_ip || !p->dst_ip || !out))
        return fail(ctx, NEXG_EINVAL, "NULL address array or output%s", nullptr);
    if (((reinterpret_cast<uint64_t>(p->src_ip) | reinterpret_cast<uint64_t>(p->dst_ip)) & 3u) != 0)
        return fail(ctx, NEXG_EINVAL, "address arrays must be 4-B aligned%s", nullptr);
    if (p->payload_len && !p->payload) return fail(ctx, NEXG_EINVAL, "NULL payload%s", nullptr);
    if (out_stride < 62u + p->payload_len)
        return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_udp6(*p, out, out_stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

static int check_ip_build(nexg_ctx* ctx, const nexg_ip_build& ip, uint64_t count, const uint8_t* out) {
    if (ip.family != 4 && ip.family != 6) return fail(ctx, NEXG_EINVAL, "IP family must be 4 or 6%s", nullptr);
    if (count && (!ip.src_ip || !ip.dst_ip || !out))
        return fail(ctx, NEXG_EINVAL, "NULL address array or output%s", nullptr);
    if (((reinterpret_cast<uint64_t>(ip.src_ip) | reinterpret_cast<uint64_t>(ip.dst_ip)) & 3u) != 0)
        return fail(ctx, NEXG_EINVAL, "address arrays must be 4-B aligned%s", nullptr);
    return NEXG_OK;
}

int nexg_build_tcp_batch(nexg_ctx* ctx, const nexg_tcp_build* p, uint8_t* out, uint32_t out_stride,
                         void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (int rc = check_ip_build(ctx, p->ip, p->count, out)) return rc;
    const uint64_t padded = (p->options_len + 3u) & ~3u;
    if (p->options_len > 40u || padded > 40u)  // builder/tcp.rs:128-135
        return fail(ctx, NEXG_ERANGE, "TCP options longer than 40 B%s", nullptr);
    const uint64_t seg = 20u + padded + p->payload_len;
    if (seg > (p->ip.family == 4 ? 65535u - 20u : 65535u))  // builder/tcp.rs:94-99, 146-152
        return fail(ctx, NEXG_ERANGE, "TCP segment length overflow%s", nullptr);
    if (p->payload_len && !p->payload) return fail(ctx, NEXG_EINVAL, "NULL payload%s", nullptr);
    const uint64_t flen = 14u + (p->ip.family == 4 ? 20u : 40u) + seg;
    if (out_stride < flen) return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_tcp(*p, out, out_stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_build_icmp_echo_batch(nexg_ctx* ctx, const nexg_icmp_echo_build* p, uint8_t* out,
                               uint32_t out_stride, void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (int rc = check_ip_build(ctx, p->ip, p->count, out)) return rc;
    const uint64_t len = 8u + (uint64_t)p->payload_len;
    if (len > (p->ip.family == 4 ? 65535u - 20u : 65535u))  // builder/icmp.rs:67-80, icmpv6.rs:72-86
        return fail(ctx, NEXG_ERANGE, "ICMP packet length overflow%s", nullptr);
    if (p->payload_len && !p->payload) return fail(ctx, NEXG_EINVAL, "NULL payload%s", nullptr);
    const uint64_t flen = 14u + (p->ip.family == 4 ? 20u : 40u) + len;
    if (out_stride < flen) return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_icmp_echo(*p, out, out_stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_build_arp_batch(nexg_ctx* ctx, const nexg_arp_build* p, uint8_t* out, uint32_t out_stride,
                         void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (p->hw_addr_len != 6)  // builder/arp.rs:101-108 BuildError::InvalidFieldLength
        return fail(ctx, NEXG_EINVAL, "InvalidFieldLength: ARP hardware address (expected 6)%s", nullptr);
    if (p->proto_addr_len != 4)  // builder/arp.rs:109-115
        return fail(ctx, NEXG_EINVAL, "InvalidFieldLength: ARP protocol address (expected 4)%s", nullptr);
    if (p->count && (!p->target_ip || !out)) return fail(ctx, NEXG_EINVAL, "NULL target array or output%s", nullptr);
    if (out_stride < 42u) return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_arp(*p, out, out_stride, static_cast<hipStream_t>(stream)), NEXG_ELAUNCH);
}

int nexg_build_ndp_ns_batch(nexg_ctx* ctx, const nexg_ndp_ns_build* p, uint8_t* out, uint32_t out_stride,
                            void* stream) {
    if (!ctx || !p) return NEXG_EINVAL;
    if (p->ip.family != 6) return fail(ctx, NEXG_EINVAL, "NDP needs IP family 6%s", nullptr);
    if (int rc = check_ip_build(ctx, p->ip, p->count, out)) return rc;
    if (out_stride < 86u) return fail(ctx, NEXG_EINVAL, "out_stride shorter than a frame%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_build_ndp_ns(*p, out, out_stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_gen_lengths(nexg_ctx* ctx, int workload, uint64_t seed, uint64_t first_index,
                     uint64_t count, uint32_t* lengths, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (workload != NEXG_WL_UDP64 && workload != NEXG_WL_IMIX) return fail(ctx, NEXG_EINVAL, "workload%s", nullptr);
    if (count && !lengths) return fail(ctx, NEXG_EINVAL, "NULL lengths%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_gen_lengths(workload, seed, first_index, count, lengths,
                                                    static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_gen_frames(nexg_ctx* ctx, int workload, uint64_t seed, uint64_t first_index,
                    uint64_t count, uint8_t* data, const uint64_t* offsets, uint32_t stride,
                    void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (workload != NEXG_WL_UDP64 && workload != NEXG_WL_IMIX) return fail(ctx, NEXG_EINVAL, "workload%s", nullptr);
    if (count && !data) return fail(ctx, NEXG_EINVAL, "NULL data%s", nullptr);
    if (!offsets && stride < (workload == NEXG_WL_UDP64 ? 64u : 1500u))
        return fail(ctx, NEXG_EINVAL, "stride shorter than the workload's frames%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_gen_frames(workload, seed, first_index, count, data, offsets,
                                                   stride, static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

int nexg_gen_udp4_params(nexg_ctx* ctx, uint64_t seed, uint64_t first_index, uint64_t count,
                         uint32_t* src_ip, uint32_t* dst_ip, uint16_t* src_port,
                         uint16_t* dst_port, uint16_t* ip_id, void* stream) {
    if (!ctx) return NEXG_EINVAL;
    if (count && (!src_ip || !dst_ip || !src_port || !dst_port || !ip_id))
        return fail(ctx, NEXG_EINVAL, "NULL output array%s", nullptr);
    DeviceGuard g(ctx);
    return hip_status(ctx, nexg::launch_gen_udp4_params(seed, first_index, count, src_ip, dst_ip,
                                                        src_port, dst_port, ip_id,
                                                        static_cast<hipStream_t>(stream)),
                      NEXG_ELAUNCH);
}

}  // extern "C"
