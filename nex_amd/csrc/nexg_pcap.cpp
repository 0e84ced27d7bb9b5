// nexg_pcap.cpp — batch ingest of capture files into the packed frame layout
// nexg_parse_batch streams (offsets without lengths: the SpanTile kernel).
//
// Replaces nex-datalink's file channel, pcap::from_file (nex-datalink/src/
// pcap.rs:95-109) driven one frame per RawReceiver::next call (pcap.rs:
// 178-190, lib.rs:363-366), with one call per batch that copies record data
// back to back into a caller buffer (pinned host memory in the e2e pipeline).
// The reference reads files through libpcap (third-party, not in the
// reference tree); the formats here are the published ones: classic pcap
// (magic a1b2c3d4 µs / a1b23c4d ns, either byte order) and pcapng (SHB, IDB
// with if_tsresol, EPB, SPB, OPB; other blocks skipped). A record yields its
// captured bytes (caplen), as libpcap's next_packet does.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/nexg.h"

struct nexg_pcap {
    FILE* f = nullptr;
    bool ng = false;
    bool swap = false;       // file byte order differs from the host's
    bool nsec = false;       // classic: nanosecond timestamps
    uint32_t linktype = 0;   // classic header / first IDB
    uint32_t snaplen = 0;
    struct Iface { uint32_t linktype; uint64_t ts_div_num; uint64_t ts_mul; bool pow2; uint32_t shift; };
    std::vector<Iface> ifaces;  // pcapng interfaces (timestamp resolution)
    std::vector<uint8_t> pending;  // a record read but not yet delivered (did not fit)
    uint64_t pending_ts = 0;
    bool has_pending = false;
    bool eof = false;
    int fatal = 0;           // sticky error of a malformed / truncated file
    char err[160] = {0};
};

namespace {

uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
uint16_t bswap16h(uint16_t v) { return (uint16_t)((v << 8) | (v >> 8)); }

int set_err(nexg_pcap* p, int rc, const char* msg) {
    snprintf(p->err, sizeof(p->err), "%s", msg);
    return rc;
}

bool read_exact(FILE* f, void* buf, size_t n) { return n == 0 || fread(buf, 1, n, f) == n; }

uint32_t rd32(const nexg_pcap* p, const uint8_t* b) {
    uint32_t v;
    memcpy(&v, b, 4);
    return p->swap ? bswap32(v) : v;
}
uint16_t rd16(const nexg_pcap* p, const uint8_t* b) {
    uint16_t v;
    memcpy(&v, b, 2);
    return p->swap ? bswap16h(v) : v;
}

// if_tsresol: MSB clear -> 10^-v s, set -> 2^-(v & 0x7f) s
nexg_pcap::Iface make_iface(uint32_t linktype, uint8_t tsresol) {
    nexg_pcap::Iface i{linktype, 1, 1, false, 0};
    if (tsresol & 0x80) {
        i.pow2 = true;
        i.shift = tsresol & 0x7f;
    } else {
        uint64_t units = 1;
        for (uint32_t k = 0; k < tsresol && k < 19; k++) units *= 10;
        // ns = ticks * 1e9 / units
        if (units <= 1000000000ull) { i.ts_mul = 1000000000ull / units; i.ts_div_num = 1; }
        else { i.ts_mul = 1; i.ts_div_num = units / 1000000000ull; }
    }
    return i;
}

uint64_t ticks_to_ns(const nexg_pcap::Iface& i, uint64_t t) {
    if (i.pow2) return (uint64_t)(((unsigned __int128)t * 1000000000ull) >> i.shift);
    return t / i.ts_div_num * i.ts_mul;
}

// Reads the next record into p->pending. Returns 1 on a record, 0 at clean
// end of file, <0 on a malformed/truncated file.
int next_record(nexg_pcap* p) {
    if (!p->ng) {
        uint8_t h[16];
        const size_t got = fread(h, 1, 16, p->f);
        if (got == 0) return 0;
        if (got != 16) return set_err(p, NEXG_EINVAL, "truncated capture file (record header)");
        const uint32_t sec = rd32(p, h), frac = rd32(p, h + 4), caplen = rd32(p, h + 8);
        if (caplen > (1u << 26)) return set_err(p, NEXG_EINVAL, "implausible record length");
        p->pending.resize(caplen);
        if (!read_exact(p->f, p->pending.data(), caplen))
            return set_err(p, NEXG_EINVAL, "truncated capture file (record data)");
        p->pending_ts = (uint64_t)sec * 1000000000ull + (uint64_t)frac * (p->nsec ? 1u : 1000u);
        return 1;
    }
    for (;;) {
        uint8_t h[8];
        const size_t got = fread(h, 1, 8, p->f);
        if (got == 0) return 0;
        if (got != 8) return set_err(p, NEXG_EINVAL, "truncated capture file (block header)");
        uint32_t type, len;
        memcpy(&type, h, 4);
        if (type == 0x0A0D0D0Au) {  // section header: byte order may change
            uint8_t bom[4];
            if (!read_exact(p->f, bom, 4)) return set_err(p, NEXG_EINVAL, "truncated section header");
            uint32_t m;
            memcpy(&m, bom, 4);
            if (m == 0x1A2B3C4Du) p->swap = false;
            else if (m == 0x4D3C2B1Au) p->swap = true;
            else return set_err(p, NEXG_EINVAL, "bad pcapng byte-order magic");
            len = rd32(p, h + 4);
            if (len < 28 || (len & 3u)) return set_err(p, NEXG_EINVAL, "bad section header length");
            if (fseek(p->f, (long)len - 12, SEEK_CUR) != 0) return set_err(p, NEXG_EINVAL, "truncated section");
            p->ifaces.clear();
            continue;
        }
        type = rd32(p, h);
        len = rd32(p, h + 4);
        if (len < 12 || (len & 3u) || len > (1u << 26)) return set_err(p, NEXG_EINVAL, "bad pcapng block length");
        std::vector<uint8_t> body(len - 8);
        if (!read_exact(p->f, body.data(), body.size())) return set_err(p, NEXG_EINVAL, "truncated pcapng block");
        const uint32_t blen = len - 12;  // body without the trailing length
        const uint8_t* b = body.data();
        if (type == 1) {  // interface description
            if (blen < 8) return set_err(p, NEXG_EINVAL, "short interface block");
            const uint32_t lt = rd16(p, b);
            uint8_t tsres = 6;
            uint32_t o = 8;
            while (o + 4 <= blen) {  // options
                const uint16_t code = rd16(p, b + o), olen = rd16(p, b + o + 2);
                if (code == 0) break;
                if (code == 9 && olen >= 1 && o + 4 < blen) tsres = b[o + 4];
                o += 4 + ((olen + 3u) & ~3u);
            }
            p->ifaces.push_back(make_iface(lt, tsres));
            if (p->ifaces.size() == 1) {
                if (p->linktype == 0) p->linktype = lt;
                p->snaplen = rd32(p, b + 4);
            }
            continue;
        }
        if (type == 6 || type == 2) {  // enhanced / obsolete packet block
            if (blen < 20) return set_err(p, NEXG_EINVAL, "short packet block");
            const uint32_t ifid = type == 6 ? rd32(p, b) : rd16(p, b);
            const uint64_t ts = ((uint64_t)rd32(p, b + 4) << 32) | rd32(p, b + 8);
            const uint32_t caplen = rd32(p, b + 12);
            if (caplen > blen - 20) return set_err(p, NEXG_EINVAL, "packet block shorter than its capture length");
            p->pending.assign(b + 20, b + 20 + caplen);
            const nexg_pcap::Iface fallback = make_iface(p->linktype, 6);
            p->pending_ts = ticks_to_ns(ifid < p->ifaces.size() ? p->ifaces[ifid] : fallback, ts);
            return 1;
        }
        if (type == 3) {  // simple packet block: no timestamp, caplen = block data
            if (blen < 4) return set_err(p, NEXG_EINVAL, "short simple packet block");
            const uint32_t orig = rd32(p, b);
            uint32_t caplen = blen - 4;
            if (orig < caplen) caplen = orig;
            const uint32_t snap = p->snaplen;
            if (snap && caplen > snap) caplen = snap;
            p->pending.assign(b + 4, b + 4 + caplen);
            p->pending_ts = 0;
            return 1;
        }
        // any other block (name resolution, statistics, custom ...): skip
    }
}

}  // namespace

extern "C" {

int nexg_pcap_open(const char* path, nexg_pcap** out) {
    if (!path || !out) return NEXG_EINVAL;
    *out = nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) return NEXG_EINVAL;
    nexg_pcap* p = new nexg_pcap();
    p->f = f;
    setvbuf(f, nullptr, _IOFBF, 1 << 22);
    uint8_t h[24];
    if (!read_exact(f, h, 4)) { nexg_pcap_close(p); return NEXG_EINVAL; }
    uint32_t m;
    memcpy(&m, h, 4);
    if (m == 0x0A0D0D0Au) {
        p->ng = true;
        rewind(f);
        // read up to the first packet so the linktype (first IDB) is known at open
        const int rc = next_record(p);
        if (rc < 0) { nexg_pcap_close(p); return NEXG_EINVAL; }
        if (rc == 1) p->has_pending = true;
        else p->eof = true;
        *out = p;
        return NEXG_OK;
    }
    if (!read_exact(f, h + 4, 20)) { nexg_pcap_close(p); return NEXG_EINVAL; }
    if (m == 0xA1B2C3D4u || m == 0xA1B23C4Du) p->swap = false;
    else if (m == 0xD4C3B2A1u || m == 0x4D3CB2A1u) p->swap = true;
    else { nexg_pcap_close(p); return NEXG_EINVAL; }
    const uint32_t mm = p->swap ? bswap32(m) : m;
    p->nsec = mm == 0xA1B23C4Du;
    p->snaplen = rd32(p, h + 16);
    p->linktype = rd32(p, h + 20) & 0x0FFFFFFFu;  // upper bits: FCS length flags
    *out = p;
    return NEXG_OK;
}

int nexg_pcap_linktype(const nexg_pcap* p) { return p ? (int)p->linktype : -1; }

const char* nexg_pcap_last_error(const nexg_pcap* p) { return p ? p->err : ""; }

int nexg_pcap_read_batch(nexg_pcap* p, uint8_t* data, uint64_t data_cap, uint64_t* offsets,
                         uint64_t max_frames, uint64_t* ts_ns, uint64_t* n_frames) {
    if (!p || !n_frames || (max_frames && (!data || !offsets))) return NEXG_EINVAL;
    uint64_t n = 0, pos = 0;
    *n_frames = 0;
    if (p->fatal) return p->fatal;
    while (n < max_frames && !p->eof) {
        if (!p->has_pending) {
            const int rc = next_record(p);
            if (rc < 0) {
                p->fatal = rc;
                if (n) break;  // deliver what is complete; the error comes with the next call
                return rc;
            }
            if (rc == 0) { p->eof = true; break; }
            p->has_pending = true;
        }
        const uint64_t len = p->pending.size();
        if (len > 65535u) return set_err(p, NEXG_ERANGE, "record longer than 65535 bytes");
        if (pos + len > data_cap) {
            if (n == 0) return set_err(p, NEXG_ERANGE, "data_cap smaller than one record");
            break;
        }
        offsets[n] = pos;
        memcpy(data + pos, p->pending.data(), len);
        if (ts_ns) ts_ns[n] = p->pending_ts;
        pos += len;
        n++;
        p->has_pending = false;
    }
    if (max_frames) offsets[n] = pos;
    *n_frames = n;
    return NEXG_OK;
}

int nexg_pcap_close(nexg_pcap* p) {
    if (!p) return NEXG_EINVAL;
    if (p->f) fclose(p->f);
    delete p;
    return NEXG_OK;
}

}  // extern "C"
