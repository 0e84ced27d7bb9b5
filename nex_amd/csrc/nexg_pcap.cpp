// nexg_pcap.cpp — batch ingest of capture files for nexg_parse_batch.
//
// Replaces nex-datalink's file channel, pcap::from_file (nex-datalink/src/
// pcap.rs:95-109) driven one frame per RawReceiver::next call (pcap.rs:
// 178-190, lib.rs:363-366), with one call per batch. The reference reads
// files through libpcap (third-party, not in the reference tree); the formats
// here are the published ones: classic pcap (magic a1b2c3d4 µs / a1b23c4d ns,
// either byte order) and pcapng (SHB, IDB with if_tsresol, EPB, SPB, OPB;
// other blocks skipped). A record yields its captured bytes (caplen), as
// libpcap's next_packet does.
//
// Two batch shapes:
//   nexg_pcap_read_batch : records copied back to back (packed, offsets only)
//   nexg_pcap_read_raw   : the file bytes themselves land in the caller's
//                          (pinned) buffer with one read; frames are described
//                          in place by offsets + lengths, so the host touches
//                          each byte once and the GPU skips the record headers.
//   nexg_pcap_map + nexg_pcap_walk_mapped : no read at all; the file is
//                          mapped (page cache) and walked in place, the caller
//                          registers the mapping for DMA and copies record
//                          regions straight to the GPU.
// All walk records in memory (scan_one); the file is read in large chunks.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <unistd.h>

#include <thread>
#include <vector>

#include "../../include/nexg.h"

namespace {

struct Iface {
    uint32_t linktype;
    bool pow2;
    uint32_t shift;     // pow2: ns = ticks * 1e9 >> shift
    uint64_t mul, div;  // else: ns = ticks / div * mul
};

// if_tsresol: MSB clear -> 10^-v s, set -> 2^-(v & 0x7f) s
Iface make_iface(uint32_t linktype, uint8_t tsresol) {
    Iface i{linktype, false, 0, 1, 1};
    if (tsresol & 0x80) {
        i.pow2 = true;
        i.shift = tsresol & 0x7f;
    } else {
        uint64_t units = 1;
        for (uint32_t k = 0; k < tsresol && k < 19; k++) units *= 10;
        if (units <= 1000000000ull) i.mul = 1000000000ull / units;
        else i.div = units / 1000000000ull;
    }
    return i;
}

uint64_t ticks_to_ns(const Iface& i, uint64_t t) {
    if (i.pow2) return (uint64_t)(((unsigned __int128)t * 1000000000ull) >> i.shift);
    return t / i.div * i.mul;
}

struct Rec {
    size_t data;  // offset of the captured bytes from the record start
    uint32_t caplen;
    uint64_t ts_ns;
};

}  // namespace

struct nexg_pcap {
    FILE* f = nullptr;
    bool ng = false;
    bool swap = false;      // file byte order differs from the host's
    bool nsec = false;      // classic: nanosecond timestamps
    uint32_t linktype = 0;  // classic header / first IDB
    uint32_t snaplen = 0;
    std::vector<Iface> ifaces;  // pcapng interfaces of the current section
    std::vector<uint8_t> buf;   // read_batch: staging of file bytes
    size_t bpos = 0, bend = 0;
    std::vector<uint8_t> carry;  // read_raw: bytes of an incomplete record
    bool file_eof = false;
    uint32_t threads = 1;  // read_raw: parallel pread pieces per chunk
    const uint8_t* map = nullptr;  // nexg_pcap_map: the file mapped read-only
    size_t map_size = 0;
    int fatal = 0;  // sticky error of a malformed / truncated file
    char err[160] = {0};
};

namespace {

int set_err(nexg_pcap* p, int rc, const char* msg) {
    snprintf(p->err, sizeof(p->err), "%s", msg);
    return rc;
}

uint32_t rd32(const nexg_pcap* p, const uint8_t* b) {
    uint32_t v;
    memcpy(&v, b, 4);
    return p->swap ? __builtin_bswap32(v) : v;
}
uint16_t rd16(const nexg_pcap* p, const uint8_t* b) {
    uint16_t v;
    memcpy(&v, b, 2);
    return p->swap ? (uint16_t)((v << 8) | (v >> 8)) : v;
}

// One record / block at b (avail bytes). Returns 1: packet (rec filled),
// 2: other block consumed, 0: incomplete (need more bytes), <0: malformed.
// *used = bytes of the record / block.
int scan_one(nexg_pcap* p, const uint8_t* b, size_t avail, size_t* used, Rec* rec) {
    if (!p->ng) {
        if (avail < 16) return 0;
        const uint32_t sec = rd32(p, b), frac = rd32(p, b + 4), caplen = rd32(p, b + 8);
        if (caplen > (1u << 26)) return set_err(p, NEXG_EINVAL, "implausible record length");
        if (avail < 16 + (size_t)caplen) return 0;
        *used = 16 + caplen;
        rec->data = 16;
        rec->caplen = caplen;
        rec->ts_ns = (uint64_t)sec * 1000000000ull + (uint64_t)frac * (p->nsec ? 1u : 1000u);
        return 1;
    }
    if (avail < 12) return 0;
    uint32_t type, len;
    memcpy(&type, b, 4);
    if (type == 0x0A0D0D0Au) {  // section header: its byte-order magic decides
        uint32_t m;
        memcpy(&m, b + 8, 4);
        if (m == 0x1A2B3C4Du) p->swap = false;
        else if (m == 0x4D3C2B1Au) p->swap = true;
        else return set_err(p, NEXG_EINVAL, "bad pcapng byte-order magic");
        len = rd32(p, b + 4);
        if (len < 28 || (len & 3u) || len > (1u << 26)) return set_err(p, NEXG_EINVAL, "bad section header length");
        if (avail < len) return 0;
        p->ifaces.clear();
        *used = len;
        return 2;
    }
    type = rd32(p, b);
    len = rd32(p, b + 4);
    if (len < 12 || (len & 3u) || len > (1u << 26)) return set_err(p, NEXG_EINVAL, "bad pcapng block length");
    if (avail < len) return 0;
    *used = len;
    const uint8_t* body = b + 8;
    const uint32_t blen = len - 12;
    if (type == 1) {  // interface description
        if (blen < 8) return set_err(p, NEXG_EINVAL, "short interface block");
        const uint32_t lt = rd16(p, body);
        uint8_t tsres = 6;
        uint32_t o = 8;
        while (o + 4 <= blen) {
            const uint16_t code = rd16(p, body + o), olen = rd16(p, body + o + 2);
            if (code == 0) break;
            if (code == 9 && olen >= 1 && o + 4 < blen) tsres = body[o + 4];
            o += 4 + ((olen + 3u) & ~3u);
        }
        p->ifaces.push_back(make_iface(lt, tsres));
        if (p->ifaces.size() == 1) {
            if (p->linktype == 0) p->linktype = lt;
            p->snaplen = rd32(p, body + 4);
        }
        return 2;
    }
    if (type == 6 || type == 2) {  // enhanced / obsolete packet block
        if (blen < 20) return set_err(p, NEXG_EINVAL, "short packet block");
        const uint32_t ifid = type == 6 ? rd32(p, body) : rd16(p, body);
        const uint64_t ts = ((uint64_t)rd32(p, body + 4) << 32) | rd32(p, body + 8);
        const uint32_t caplen = rd32(p, body + 12);
        if (caplen > blen - 20) return set_err(p, NEXG_EINVAL, "packet block shorter than its capture length");
        rec->data = 28;
        rec->caplen = caplen;
        rec->ts_ns = ticks_to_ns(ifid < p->ifaces.size() ? p->ifaces[ifid] : make_iface(p->linktype, 6), ts);
        return 1;
    }
    if (type == 3) {  // simple packet block: no timestamp; caplen = min(orig, data, snaplen)
        if (blen < 4) return set_err(p, NEXG_EINVAL, "short simple packet block");
        const uint32_t orig = rd32(p, body);
        uint32_t caplen = blen - 4;
        if (orig < caplen) caplen = orig;
        if (p->snaplen && caplen > p->snaplen) caplen = p->snaplen;
        rec->data = 12;
        rec->caplen = caplen;
        rec->ts_ns = 0;
        return 1;
    }
    return 2;  // name resolution, statistics, custom ...: skipped
}

// read_raw's file read of `want` bytes into dst with up to p->threads
// parallel preads of >= 4-MiB pieces (one thread copies ~10 GB/s out of the
// page cache; the pinned staging buffer is the destination either way). The
// FILE position is moved past what was read. Returns the bytes read.
size_t read_parallel(nexg_pcap* p, uint8_t* dst, size_t want) {
    constexpr size_t kPiece = 4u << 20;
    const off_t base = ftello(p->f);
    const int fd = fileno(p->f);
    size_t pieces = (want + kPiece - 1) / kPiece;
    if (pieces > p->threads) pieces = p->threads;
    const size_t per = (want + pieces - 1) / pieces;
    std::vector<size_t> got(pieces, 0);
    auto work = [&](size_t k) {
        const size_t a = k * per, b = a + per < want ? a + per : want;
        size_t pos = a;
        while (pos < b) {
            const size_t n = b - pos < kPiece ? b - pos : kPiece;
            const ssize_t r = pread(fd, dst + pos, n, base + (off_t)pos);
            if (r <= 0) break;
            pos += (size_t)r;
        }
        got[k] = pos - a;
    };
    std::vector<std::thread> pool;
    for (size_t k = 1; k < pieces; k++) pool.emplace_back(work, k);
    work(0);
    for (auto& t : pool) t.join();
    size_t total = 0;  // contiguous prefix: a short piece means the file ended there
    for (size_t k = 0; k < pieces; k++) {
        total += got[k];
        if (got[k] < (k * per + per < want ? per : want - k * per)) break;
    }
    fseeko(p->f, base + (off_t)total, SEEK_SET);
    return total;
}

// read_batch staging: try to make at least `need` unread bytes available
void refill(nexg_pcap* p, size_t need) {
    if (p->bend - p->bpos >= need || p->file_eof) return;
    const size_t left = p->bend - p->bpos;
    if (p->bpos) memmove(p->buf.data(), p->buf.data() + p->bpos, left);
    p->bpos = 0;
    p->bend = left;
    size_t want = need > (4u << 20) ? need : (4u << 20);
    if (p->buf.size() < want) p->buf.resize(want);
    while (p->bend < p->buf.size()) {
        const size_t got = fread(p->buf.data() + p->bend, 1, p->buf.size() - p->bend, p->f);
        p->bend += got;
        if (got == 0) {
            p->file_eof = true;
            break;
        }
    }
}

// Classic-pcap record walk of buf[0, have) split over `threads` threads.
// Chunk k > 0 starts at the first position whose header is plausible
// (caplen <= snaplen, orig_len >= caplen, sub-second field in range) and
// chains to further plausible headers; each thread walks its chunk to the
// first record that starts at or past the chunk end. The chunks are stitched
// where the previous walk ended exactly where the next one began; any
// disagreement (a header look-alike inside a payload) re-walks that chunk
// from the previous end, so the result always equals the sequential walk.
// Returns records found (<= max_frames) and *end = bytes described, or -1
// when a malformed record needs the sequential walk's error path.
struct WalkPart {
    std::vector<uint64_t> offs;
    std::vector<uint32_t> lens;
    std::vector<uint64_t> ts;
    size_t begin = 0, end = 0;  // first record start, first start past the chunk (or the incomplete tail)
    bool bad = false;
};

bool classic_plausible(const nexg_pcap* p, const uint8_t* b, size_t avail) {
    if (avail < 16) return false;
    const uint32_t frac = rd32(p, b + 4), caplen = rd32(p, b + 8), orig = rd32(p, b + 12);
    const uint32_t snap = p->snaplen ? p->snaplen : 262144u;
    return caplen <= snap && orig >= caplen && frac < (p->nsec ? 1000000000u : 1000000u);
}

void walk_classic(const nexg_pcap* p, const uint8_t* buf, size_t have, size_t from, size_t stop, bool want_ts,
                  WalkPart& w) {
    size_t pos = from;
    w.begin = from;
    while (pos < stop) {
        if (have - pos < 16) break;
        const uint32_t caplen = rd32(p, buf + pos + 8);
        if (caplen > (1u << 26)) { w.bad = true; break; }
        if (have - pos < 16 + (size_t)caplen) break;
        w.offs.push_back(pos + 16);
        w.lens.push_back(caplen);
        if (want_ts)
            w.ts.push_back((uint64_t)rd32(p, buf + pos) * 1000000000ull +
                           (uint64_t)rd32(p, buf + pos + 4) * (p->nsec ? 1u : 1000u));
        pos += 16 + caplen;
    }
    w.end = pos;
}

// The walk is a dependent chain of header loads (each record's length gives
// the next header's address), so one chain per thread is memory-latency
// bound; each thread walks kChains chunks interleaved, one header of each per
// step, to keep that many cache misses in flight.
constexpr size_t kChains = 8;

void walk_interleaved(const nexg_pcap* p, const uint8_t* buf, size_t have, const size_t* from, const size_t* stop,
                      bool want_ts, WalkPart* w, size_t m) {
    size_t pos[kChains];
    bool live[kChains];
    size_t active = 0;
    for (size_t j = 0; j < m; j++) {
        pos[j] = from[j];
        w[j].begin = from[j];
        w[j].end = from[j];  // a chain that never starts describes nothing: it ends where it began
        live[j] = pos[j] < stop[j];
        active += live[j];
    }
    while (active) {
        for (size_t j = 0; j < m; j++) {
            if (!live[j]) continue;
            const size_t q = pos[j];
            bool go = q < stop[j] && have - q >= 16;
            uint32_t caplen = 0;
            if (go) {
                caplen = rd32(p, buf + q + 8);
                if (caplen > (1u << 26)) { w[j].bad = true; go = false; }
                else if (have - q < 16 + (size_t)caplen) go = false;
            }
            if (!go) {
                live[j] = false;
                active--;
                w[j].end = q;
                continue;
            }
            w[j].offs.push_back(q + 16);
            w[j].lens.push_back(caplen);
            if (want_ts)
                w[j].ts.push_back((uint64_t)rd32(p, buf + q) * 1000000000ull +
                                  (uint64_t)rd32(p, buf + q + 4) * (p->nsec ? 1u : 1000u));
            pos[j] = q + 16 + caplen;
        }
    }
}

int64_t parallel_walk(nexg_pcap* p, const uint8_t* buf, size_t have, uint64_t max_frames, uint64_t* offsets,
                      uint32_t* lengths, uint64_t* ts_ns, size_t* end) {
    const size_t T = p->threads * kChains;  // chunks: kChains per thread
    const size_t per = (have + T - 1) / T;
    std::vector<WalkPart> parts(T);
    auto start_of = [&](size_t k) {  // chunk k's first plausible header that chains 4 deep (or to the end)
        const size_t a = k * per, b = a + per < have ? a + per : have;
        size_t s = a;
        if (k > 0) {
            for (; s < b; s++) {
                size_t q = s;
                int depth = 0;
                while (depth < 4 && classic_plausible(p, buf + q, have - q)) {
                    q += 16 + (size_t)rd32(p, buf + q + 8);
                    depth++;
                    if (q >= have) break;
                }
                if (depth == 4 || (depth > 0 && q >= have)) break;
            }
        }
        return s;
    };
    auto work = [&](size_t t) {
        size_t from[kChains], stop[kChains];
        for (size_t j = 0; j < kChains; j++) {
            const size_t k = t * kChains + j, a = k * per;
            if (a >= have) {
                from[j] = stop[j] = have;
                continue;
            }
            stop[j] = a + per < have ? a + per : have;
            from[j] = start_of(k);
        }
        walk_interleaved(p, buf, have, from, stop, ts_ns != nullptr, &parts[t * kChains], kChains);
    };
    std::vector<std::thread> pool;
    for (size_t t = 1; t < p->threads; t++) pool.emplace_back(work, t);
    work(0);
    for (auto& t : pool) t.join();
    // stitch; re-walk a chunk whose start disagrees with the previous end
    for (size_t k = 1; k < T; k++) {
        if (parts[k - 1].bad) return -1;
        if (parts[k].begin != parts[k - 1].end) {
            const size_t stop = (k + 1) * per < have ? (k + 1) * per : have;
            parts[k] = WalkPart{};
            walk_classic(p, buf, have, parts[k - 1].end, stop > parts[k - 1].end ? stop : parts[k - 1].end,
                         ts_ns != nullptr, parts[k]);
        }
    }
    if (parts[T - 1].bad) return -1;
    // concatenate (up to max_frames), in parallel
    std::vector<uint64_t> first(T + 1, 0);
    for (size_t k = 0; k < T; k++) first[k + 1] = first[k] + parts[k].offs.size();
    const uint64_t n = first[T] < max_frames ? first[T] : max_frames;
    auto copy = [&](size_t k) {
        if (first[k] >= n) return;
        const uint64_t m = (first[k + 1] < n ? first[k + 1] : n) - first[k];
        memcpy(offsets + first[k], parts[k].offs.data(), m * 8);
        memcpy(lengths + first[k], parts[k].lens.data(), m * 4);
        if (ts_ns) memcpy(ts_ns + first[k], parts[k].ts.data(), m * 8);
    };
    auto copy_chunks = [&](size_t t) {
        for (size_t j = 0; j < kChains; j++) copy(t * kChains + j);
    };
    pool.clear();
    for (size_t t = 1; t < p->threads; t++) pool.emplace_back(copy_chunks, t);
    copy_chunks(0);
    for (auto& t : pool) t.join();
    *end = n < first[T] ? (size_t)(offsets[n - 1] + lengths[n - 1]) : parts[T - 1].end;
    if (n == 0) *end = 0;
    return (int64_t)n;
}

// Records of buf[0, have): the parallel classic walk when it applies, else
// scan_one in sequence; offsets / lengths into buf, *pos = bytes described.
// Returns 0, or the error of a malformed record met before any frame.
int walk_records(nexg_pcap* p, const uint8_t* buf, size_t have, uint64_t max_frames, uint64_t* offsets,
                 uint32_t* lengths, uint64_t* ts_ns, uint64_t* n_out, size_t* pos_out) {
    uint64_t n = 0;
    size_t pos = 0;
    bool walked = false;
    if (!p->ng && have >= (8u << 20)) {  // classic pcap: chunked walk (kChains per thread, threads in parallel)
        size_t end = 0;
        const int64_t got = parallel_walk(p, buf, have, max_frames, offsets, lengths, ts_ns, &end);
        if (got >= 0) {
            n = (uint64_t)got;
            pos = end;
            walked = true;
        }  // else: a malformed record; the sequential walk below reports it
    }
    while (!walked && n < max_frames) {
        size_t used = 0;
        Rec r;
        const int rc = scan_one(p, buf + pos, have - pos, &used, &r);
        if (rc == 0) break;
        if (rc < 0) {
            p->fatal = rc;
            if (n) break;
            return rc;
        }
        if (rc == 1) {  // > 65535 B passes through (NEXG_ERR_BAD_EXTENT in the parse)
            offsets[n] = pos + r.data;
            lengths[n] = r.caplen;
            if (ts_ns) ts_ns[n] = r.ts_ns;
            n++;
        }
        pos += used;
    }
    *n_out = n;
    *pos_out = pos;
    return 0;
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
    uint8_t h[24];
    const size_t got = fread(h, 1, 24, f);
    uint32_t m = 0;
    if (got >= 4) memcpy(&m, h, 4);
    if (m == 0x0A0D0D0Au) {
        p->ng = true;
        rewind(f);
        // walk up to the first packet so the linktype (first IDB) is known now;
        // the bytes read so far become the carry of the first read
        for (;;) {
            refill(p, 12);
            size_t used = 0;
            Rec r;
            const int rc = scan_one(p, p->buf.data() + p->bpos, p->bend - p->bpos, &used, &r);
            if (rc == 0 && !p->file_eof) { refill(p, p->bend - p->bpos + 65536); continue; }
            if (rc < 0 || (rc == 0 && p->bend > p->bpos)) { nexg_pcap_close(p); return NEXG_EINVAL; }
            if (rc != 2) break;  // a packet (left for the first read) or an empty file
            p->bpos += used;
        }
        p->carry.assign(p->buf.begin() + p->bpos, p->buf.begin() + p->bend);
        p->bpos = p->bend = 0;
        *out = p;
        return NEXG_OK;
    }
    if (got != 24) { nexg_pcap_close(p); return NEXG_EINVAL; }
    if (m == 0xA1B2C3D4u || m == 0xA1B23C4Du) p->swap = false;
    else if (m == 0xD4C3B2A1u || m == 0x4D3CB2A1u) p->swap = true;
    else { nexg_pcap_close(p); return NEXG_EINVAL; }
    const uint32_t mm = p->swap ? __builtin_bswap32(m) : m;
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
    if (!p->carry.empty()) {  // bytes staged by open or by read_raw come first
        std::vector<uint8_t> staged(p->carry.begin(), p->carry.end());
        staged.insert(staged.end(), p->buf.begin() + p->bpos, p->buf.begin() + p->bend);
        p->buf.swap(staged);
        p->bpos = 0;
        p->bend = p->buf.size();
        p->carry.clear();
    }
    while (n < max_frames) {
        refill(p, 16);
        size_t used = 0;
        Rec r;
        const int rc = scan_one(p, p->buf.data() + p->bpos, p->bend - p->bpos, &used, &r);
        if (rc == 0) {
            if (p->file_eof) {
                if (p->bend > p->bpos) {  // a torn record at the end of the file
                    p->fatal = set_err(p, NEXG_EINVAL, "truncated capture file");
                    if (n) break;
                    return p->fatal;
                }
                break;  // clean end of file
            }
            refill(p, p->bend - p->bpos + 65536);  // the record is larger than what is staged
            continue;
        }
        if (rc < 0) {
            p->fatal = rc;
            if (n) break;  // deliver what is complete; the error comes with the next call
            return rc;
        }
        if (rc == 2) {
            p->bpos += used;
            continue;
        }
        // a record longer than 65535 B (loopback / GRO captures) passes through:
        // the parse kernels report it per frame as NEXG_ERR_BAD_EXTENT
        if (pos + r.caplen > data_cap) {
            if (n == 0) return set_err(p, NEXG_ERANGE, "data_cap smaller than one record");
            break;
        }
        offsets[n] = pos;
        memcpy(data + pos, p->buf.data() + p->bpos + r.data, r.caplen);
        if (ts_ns) ts_ns[n] = r.ts_ns;
        pos += r.caplen;
        n++;
        p->bpos += used;
    }
    if (max_frames) offsets[n] = pos;
    *n_frames = n;
    return NEXG_OK;
}

int nexg_pcap_read_raw(nexg_pcap* p, uint8_t* buf, uint64_t cap, uint64_t* offsets,
                       uint32_t* lengths, uint64_t max_frames, uint64_t* ts_ns, uint64_t* n_frames,
                       uint64_t* bytes_used) {
    if (!p || !n_frames || !bytes_used || !buf || !max_frames || !offsets || !lengths) return NEXG_EINVAL;
    *n_frames = 0;
    *bytes_used = 0;
    if (p->fatal) return p->fatal;
    if (p->bend > p->bpos) {  // bytes staged by read_batch come first
        p->carry.insert(p->carry.end(), p->buf.begin() + p->bpos, p->buf.begin() + p->bend);
        p->bpos = p->bend = 0;
    }
    // carried bytes first (possibly more than fit: the rest stays carried)
    size_t have = p->carry.size() < cap ? p->carry.size() : (size_t)cap;
    if (have) memcpy(buf, p->carry.data(), have);
    p->carry.erase(p->carry.begin(), p->carry.begin() + have);
    if (p->threads > 1 && have < cap && p->carry.empty() && !p->file_eof) {
        const size_t got = read_parallel(p, buf + have, cap - have);
        if (got < cap - have) p->file_eof = true;
        have += got;
    }
    while (have < cap && p->carry.empty() && !p->file_eof) {
        // 4-MiB reads: one huge read() into pinned memory measured ~2x slower
        const size_t want = cap - have < (4u << 20) ? cap - have : (4u << 20);
        const size_t got = fread(buf + have, 1, want, p->f);
        have += got;
        if (got == 0) p->file_eof = true;
    }
    uint64_t n = 0;
    size_t pos = 0;
    const int wrc = walk_records(p, buf, have, max_frames, offsets, lengths, ts_ns, &n, &pos);
    if (wrc) return wrc;
    if (pos < have) {  // an incomplete record, or records past max_frames: next call
        if (n == 0 && pos == 0 && p->file_eof && p->carry.empty() && have < cap)
            return p->fatal = set_err(p, NEXG_EINVAL, "truncated capture file");
        // every byte not described goes back in front of the carry, so a retry
        // (e.g. with a larger buffer after NEXG_ERANGE) resumes at this record
        p->carry.insert(p->carry.begin(), buf + pos, buf + have);
        if (n == 0 && pos == 0) return set_err(p, NEXG_ERANGE, "buffer smaller than one record");
    }
    *n_frames = n;
    *bytes_used = pos;
    return NEXG_OK;
}

int nexg_pcap_map(nexg_pcap* p, const uint8_t** data, uint64_t* size, uint64_t* first) {
    if (!p || !data || !size || !first) return NEXG_EINVAL;
    if (!p->map) {
        struct stat st;
        const int fd = fileno(p->f);
        if (fstat(fd, &st) != 0) return set_err(p, NEXG_EINVAL, "fstat failed");
        if (st.st_size > 0) {
            // no MAP_POPULATE: a capture may be far larger than host memory;
            // pages come in as the walk (or the caller's DMA registration of
            // a window) reaches them, read ahead sequentially
            void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
            if (m == MAP_FAILED) return set_err(p, NEXG_ENOMEM, "mmap failed");
            madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL);
            p->map = static_cast<const uint8_t*>(m);
        }
        p->map_size = (size_t)st.st_size;
    }
    *data = p->map;
    *size = p->map_size;
    *first = p->ng ? 0u : 24u;  // pcapng: the blocks from the section header on
    return NEXG_OK;
}

int nexg_pcap_walk_mapped(nexg_pcap* p, uint64_t from, uint64_t max_bytes, uint64_t* offsets,
                          uint32_t* lengths, uint64_t max_frames, uint64_t* ts_ns, uint64_t* n_frames,
                          uint64_t* next) {
    if (!p || !n_frames || !next || !max_frames || !offsets || !lengths) return NEXG_EINVAL;
    *n_frames = 0;
    *next = from;
    if (!p->map && p->map_size == 0) return set_err(p, NEXG_EINVAL, "walk_mapped before nexg_pcap_map");
    if (from > p->map_size) return set_err(p, NEXG_EINVAL, "offset past the end of the file");
    if (p->fatal) return p->fatal;
    const size_t left = p->map_size - (size_t)from;
    const size_t have = max_bytes < left ? (size_t)max_bytes : left;
    if (have == 0) return NEXG_OK;  // end of file
    uint64_t n = 0;
    size_t pos = 0;
    const int rc = walk_records(p, p->map + from, have, max_frames, offsets, lengths, ts_ns, &n, &pos);
    if (rc) return rc;
    if (n == 0 && pos == 0) {  // not even one record in the window
        if (have == left) return p->fatal = set_err(p, NEXG_EINVAL, "truncated capture file");
        return set_err(p, NEXG_ERANGE, "max_bytes smaller than one record");
    }
    *n_frames = n;
    *next = from + pos;
    return NEXG_OK;
}

int nexg_pcap_set_read_threads(nexg_pcap* p, uint32_t threads) {
    if (!p || threads == 0 || threads > 64) return NEXG_EINVAL;
    p->threads = threads;
    return NEXG_OK;
}

int nexg_pcap_close(nexg_pcap* p) {
    if (!p) return NEXG_EINVAL;
    if (p->map) munmap(const_cast<uint8_t*>(p->map), p->map_size);
    if (p->f) fclose(p->f);
    delete p;
    return NEXG_OK;
}

}  // extern "C"
