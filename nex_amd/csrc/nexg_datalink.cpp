// nexg_datalink.cpp — live batch rx / tx for the GPU parse path (SURVEY.md
// 8(f)2; include/nexg.h "live datalink batch rx / tx").
//
// The reference's Linux channel (nex-datalink/src/linux.rs:102-218) opens one
// AF_PACKET SOCK_RAW socket per channel (ETH_P_ALL, bound to the interface,
// optional promiscuous membership and PACKET_FANOUT group, O_NONBLOCK) and
// moves ONE frame per system call: poll + recvfrom into a 4096-B read buffer
// (linux.rs:356-397), poll + sendto (linux.rs:302-346). A batch engine that
// parses 100 Gpkt/s cannot be fed that way, so here the same socket setup
// feeds whole batches:
//   rx, NEXG_RX_RING : a TPACKET_V3 mmap ring; the kernel fills fixed-size
//                      blocks and retires them (full or after the block
//                      timeout); a batch call walks every retired block and
//                      copies the frames into the caller's pinned buffer in
//                      the packed layout (offsets only) the span kernel reads.
//   rx, NEXG_RX_MMSG : recvmmsg into read_buffer_size slots, then packed.
//   tx               : sendmmsg, up to 1024 frames per system call.
// Frames are truncated to read_buffer_size, as recvfrom into the reference's
// read buffer truncates them (lib.rs:229-240, linux.rs:388-390).
#include <arpa/inet.h>
#include <errno.h>
#include <linux/if_packet.h>
#include <net/ethernet.h>
#include <net/if.h>
#include <poll.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <vector>

#include "../../include/nexg.h"

struct nexg_rx {
    int fd = -1;
    nexg_rx_config cfg{};
    uint8_t* ring = nullptr;  // TPACKET_V3: ring_blocks x ring_block_size
    size_t ring_bytes = 0;
    uint32_t block = 0;     // current block
    uint32_t pkt = 0;       // next packet of the current block
    std::vector<uint8_t> slots;  // NEXG_RX_MMSG staging
};

struct nexg_tx {
    int fd = -1;
    sockaddr_ll addr{};
};

namespace {

int errno_status(int e) { return (e == EPERM || e == EACCES) ? NEXG_EPERM : NEXG_EIO; }

int64_t now_ms() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

// linux.rs:102-197: socket, bind to the interface, promiscuous membership
int open_bound(const char* ifname, int* fd_out, sockaddr_ll* addr_out) {
    const unsigned idx = if_nametoindex(ifname);
    if (idx == 0) return NEXG_EINVAL;
    const int fd = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
    if (fd < 0) return errno_status(errno);
    sockaddr_ll a{};
    a.sll_family = AF_PACKET;
    a.sll_protocol = htons(ETH_P_ALL);
    a.sll_ifindex = (int)idx;
    *fd_out = fd;
    *addr_out = a;
    return NEXG_OK;
}

}  // namespace

extern "C" {

void nexg_rx_config_default(nexg_rx_config* c) {
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->read_buffer_size = 4096;  // Config::default (lib.rs:229-240)
    c->read_timeout_ms = -1;     // read_timeout: None -> wait
    c->promiscuous = 1;          // Config::default promiscuous: true
    c->mode = NEXG_RX_RING;
    c->ring_block_size = 1u << 20;
    c->ring_blocks = 64;
    c->ring_block_tov_ms = 2;
}

int nexg_rx_open(const char* ifname, const nexg_rx_config* cfg_in, nexg_rx** out) {
    if (!ifname || !out) return NEXG_EINVAL;
    *out = nullptr;
    nexg_rx_config cfg;
    if (cfg_in) cfg = *cfg_in;
    else nexg_rx_config_default(&cfg);
    if (cfg.read_buffer_size == 0 || cfg.read_buffer_size > 65535 || cfg.mode > NEXG_RX_MMSG) return NEXG_EINVAL;
    if (cfg.mode == NEXG_RX_RING &&
        (cfg.ring_blocks == 0 || cfg.ring_block_size < 4096 || (cfg.ring_block_size & 4095u) != 0))
        return NEXG_EINVAL;
    int fd;
    sockaddr_ll a;
    int rc = open_bound(ifname, &fd, &a);
    if (rc) return rc;
    nexg_rx* rx = new nexg_rx();
    rx->fd = fd;
    rx->cfg = cfg;
    auto fail = [&](int code) {
        nexg_rx_close(rx);
        return code;
    };
    if (cfg.mode == NEXG_RX_RING) {  // the ring is set up before bind, so no frame is missed
        int v = TPACKET_V3;
        if (setsockopt(fd, SOL_PACKET, PACKET_VERSION, &v, sizeof(v)) < 0) return fail(errno_status(errno));
        tpacket_req3 req{};
        req.tp_block_size = cfg.ring_block_size;
        req.tp_block_nr = cfg.ring_blocks;
        req.tp_frame_size = 2048;  // v3 packs frames by size; the field only has to divide the block
        req.tp_frame_nr = (unsigned)((uint64_t)cfg.ring_block_size * cfg.ring_blocks / req.tp_frame_size);
        req.tp_retire_blk_tov = cfg.ring_block_tov_ms;
        if (setsockopt(fd, SOL_PACKET, PACKET_RX_RING, &req, sizeof(req)) < 0) return fail(errno_status(errno));
        rx->ring_bytes = (size_t)cfg.ring_block_size * cfg.ring_blocks;
        void* m = mmap(nullptr, rx->ring_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m == MAP_FAILED) {
            rx->ring_bytes = 0;
            return fail(NEXG_EIO);
        }
        rx->ring = static_cast<uint8_t*>(m);
    }
    if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0) return fail(errno_status(errno));
    if (cfg.promiscuous) {  // linux.rs:131-151
        packet_mreq mr{};
        mr.mr_ifindex = a.sll_ifindex;
        mr.mr_type = PACKET_MR_PROMISC;
        if (setsockopt(fd, SOL_PACKET, PACKET_ADD_MEMBERSHIP, &mr, sizeof(mr)) < 0) return fail(errno_status(errno));
    }
    if (cfg.fanout) {  // linux.rs:154-193: group_id | (type | flags) << 16
        const unsigned arg = (cfg.fanout_group & 0xFFFFu) | (cfg.fanout_type << 16);
        if (setsockopt(fd, SOL_PACKET, PACKET_FANOUT, &arg, sizeof(arg)) < 0) return fail(errno_status(errno));
    }
    if (cfg.mode == NEXG_RX_MMSG) {
        // the socket queue is the only buffer here: size it like the ring
        // (SO_RCVBUFFORCE needs CAP_NET_ADMIN; SO_RCVBUF is capped at rmem_max)
        const int want = (int)((uint64_t)cfg.ring_block_size * cfg.ring_blocks < (1u << 30)
                                   ? (uint64_t)cfg.ring_block_size * cfg.ring_blocks : (1u << 30));
        if (setsockopt(fd, SOL_SOCKET, SO_RCVBUFFORCE, &want, sizeof(want)) < 0)
            (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &want, sizeof(want));
        rx->slots.resize((size_t)1024 * cfg.read_buffer_size);
    }
    *out = rx;
    return NEXG_OK;
}

int nexg_tpacket3_walk(const uint8_t* block, uint64_t block_bytes, uint32_t first, uint32_t snap, uint32_t flags,
                       uint8_t* data, uint64_t data_cap, uint64_t* pos, uint64_t* offsets, uint64_t max_frames,
                       uint64_t* ts_ns, uint64_t* n, uint32_t* next_pkt) {
    if (!block || !pos || !offsets || !n || !next_pkt || (max_frames && !data)) return NEXG_EINVAL;
    if (block_bytes < sizeof(tpacket_block_desc)) return NEXG_EINVAL;
    const tpacket_block_desc* bd = reinterpret_cast<const tpacket_block_desc*>(block);
    const uint32_t num = bd->hdr.bh1.num_pkts;
    uint64_t off = bd->hdr.bh1.offset_to_first_pkt;
    uint32_t k = 0;
    // headers are chained by tp_next_offset; skip the `first` already taken
    for (; k < num; k++) {
        if (off + sizeof(tpacket3_hdr) > block_bytes) return NEXG_EINVAL;
        const tpacket3_hdr* h = reinterpret_cast<const tpacket3_hdr*>(block + off);
        if (k >= first) {
            if (*n >= max_frames) break;
            const uint32_t cap = h->tp_snaplen < snap ? h->tp_snaplen : snap;
            if ((uint64_t)h->tp_mac + h->tp_snaplen > block_bytes - off) return NEXG_EINVAL;
            const sockaddr_ll* sll = reinterpret_cast<const sockaddr_ll*>(
                block + off + TPACKET_ALIGN(sizeof(tpacket3_hdr)));
            const bool skip = (flags & NEXG_RX_SKIP_OUTGOING) && sll->sll_pkttype == PACKET_OUTGOING;
            if (!skip) {
                if (*pos + cap > data_cap) break;
                memcpy(data + *pos, block + off + h->tp_mac, cap);
                offsets[*n] = *pos;
                if (ts_ns) ts_ns[*n] = (uint64_t)h->tp_sec * 1000000000ull + h->tp_nsec;
                *pos += cap;
                (*n)++;
            }
        }
        if (h->tp_next_offset == 0 && k + 1 < num) return NEXG_EINVAL;
        off += h->tp_next_offset;
    }
    *next_pkt = k;
    return NEXG_OK;
}

int nexg_rx_next_batch(nexg_rx* rx, uint8_t* data, uint64_t data_cap, uint64_t* offsets, uint64_t max_frames,
                       uint64_t* ts_ns, uint64_t* n_frames) {
    if (!rx || !n_frames || (max_frames && (!data || !offsets))) return NEXG_EINVAL;
    *n_frames = 0;
    if (max_frames == 0) return NEXG_OK;
    uint64_t n = 0, pos = 0;
    const int64_t deadline = rx->cfg.read_timeout_ms < 0 ? -1 : now_ms() + rx->cfg.read_timeout_ms;
    if (rx->cfg.mode == NEXG_RX_RING) {
        for (;;) {
            // take every retired block in ring order
            while (n < max_frames) {
                uint8_t* blk = rx->ring + (size_t)rx->block * rx->cfg.ring_block_size;
                tpacket_block_desc* bd = reinterpret_cast<tpacket_block_desc*>(blk);
                std::atomic_thread_fence(std::memory_order_acquire);
                if (!(__atomic_load_n(&bd->hdr.bh1.block_status, __ATOMIC_ACQUIRE) & TP_STATUS_USER)) break;
                uint32_t next = 0;
                const int rc = nexg_tpacket3_walk(blk, rx->cfg.ring_block_size, rx->pkt, rx->cfg.read_buffer_size,
                                                  rx->cfg.flags, data, data_cap, &pos, offsets, max_frames, ts_ns,
                                                  &n, &next);
                if (rc) return rc;
                if (next < bd->hdr.bh1.num_pkts) {  // the batch is full: resume here next call
                    rx->pkt = next;
                    if (n == 0) return NEXG_ERANGE;  // not even the next frame fits data_cap: never spin on it
                    break;
                }
                __atomic_store_n(&bd->hdr.bh1.block_status, (uint32_t)TP_STATUS_KERNEL, __ATOMIC_RELEASE);
                rx->pkt = 0;
                rx->block = (rx->block + 1) % rx->cfg.ring_blocks;
            }
            if (n > 0 || n >= max_frames) break;
            int wait = -1;
            if (deadline >= 0) {
                const int64_t left = deadline - now_ms();
                if (left <= 0) break;
                wait = (int)left;
            }
            pollfd p{rx->fd, POLLIN | POLLERR, 0};
            const int pr = poll(&p, 1, wait);
            if (pr < 0 && errno != EINTR) return NEXG_EIO;
            if (pr == 0) break;
        }
    } else {
        const uint32_t S = rx->cfg.read_buffer_size;
        if (data_cap < S) return NEXG_ERANGE;  // no slot ever fits: fail instead of polling a readable socket forever
        std::vector<mmsghdr> msgs(1024);
        std::vector<iovec> iov(1024);
        std::vector<sockaddr_ll> from(1024);
        for (;;) {
            while (n < max_frames) {
                const uint64_t want = max_frames - n < 1024 ? max_frames - n : 1024;
                for (uint64_t k = 0; k < want; k++) {
                    iov[k] = {rx->slots.data() + k * S, S};
                    msgs[k] = {};
                    msgs[k].msg_hdr.msg_iov = &iov[k];
                    msgs[k].msg_hdr.msg_iovlen = 1;
                    msgs[k].msg_hdr.msg_name = &from[k];
                    msgs[k].msg_hdr.msg_namelen = sizeof(sockaddr_ll);
                }
                // the data_cap bound: never take more frames than surely fit
                uint64_t fit = (data_cap - pos) / S;
                const uint64_t take = fit < want ? fit : want;
                if (take == 0) break;
                const int got = recvmmsg(rx->fd, msgs.data(), (unsigned)take, MSG_DONTWAIT, nullptr);
                if (got < 0) {
                    if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) break;
                    return NEXG_EIO;
                }
                timespec ts;
                clock_gettime(CLOCK_REALTIME, &ts);
                for (int k = 0; k < got; k++) {
                    if ((rx->cfg.flags & NEXG_RX_SKIP_OUTGOING) && from[k].sll_pkttype == PACKET_OUTGOING) continue;
                    const uint32_t len = msgs[k].msg_len < S ? msgs[k].msg_len : S;
                    memcpy(data + pos, rx->slots.data() + (size_t)k * S, len);
                    offsets[n] = pos;
                    if (ts_ns) ts_ns[n] = (uint64_t)ts.tv_sec * 1000000000ull + ts.tv_nsec;
                    pos += len;
                    n++;
                }
                if ((uint64_t)got < take) break;
            }
            if (n > 0) break;
            int wait = -1;
            if (deadline >= 0) {
                const int64_t left = deadline - now_ms();
                if (left <= 0) break;
                wait = (int)left;
            }
            pollfd p{rx->fd, POLLIN | POLLERR, 0};
            const int pr = poll(&p, 1, wait);
            if (pr < 0 && errno != EINTR) return NEXG_EIO;
            if (pr == 0) break;
        }
    }
    offsets[n] = pos;
    *n_frames = n;
    return NEXG_OK;
}

int nexg_rx_stats(nexg_rx* rx, uint64_t* packets, uint64_t* drops) {
    if (!rx || !packets || !drops) return NEXG_EINVAL;
    tpacket_stats_v3 st{};
    socklen_t len = sizeof(st);
    if (getsockopt(rx->fd, SOL_PACKET, PACKET_STATISTICS, &st, &len) < 0) return NEXG_EIO;
    *packets = st.tp_packets;
    *drops = st.tp_drops;
    return NEXG_OK;
}

int nexg_rx_close(nexg_rx* rx) {
    if (!rx) return NEXG_EINVAL;
    if (rx->ring) munmap(rx->ring, rx->ring_bytes);
    if (rx->fd >= 0) close(rx->fd);
    delete rx;
    return NEXG_OK;
}

int nexg_tx_open(const char* ifname, nexg_tx** out) {
    if (!ifname || !out) return NEXG_EINVAL;
    *out = nullptr;
    int fd;
    sockaddr_ll a;
    const int rc = open_bound(ifname, &fd, &a);
    if (rc) return rc;
    if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) < 0) {
        const int e = errno_status(errno);
        close(fd);
        return e;
    }
    nexg_tx* tx = new nexg_tx();
    tx->fd = fd;
    tx->addr = a;
    *out = tx;
    return NEXG_OK;
}

int nexg_tx_send_batch(nexg_tx* tx, const uint8_t* data, const uint64_t* offsets, const uint32_t* lengths,
                       uint32_t stride, uint64_t count, uint64_t* n_sent) {
    if (!tx || !n_sent || (count && !data) || (!offsets && stride == 0 && count)) return NEXG_EINVAL;
    *n_sent = 0;
    std::vector<mmsghdr> msgs(1024);
    std::vector<iovec> iov(1024);
    uint64_t done = 0;
    while (done < count) {
        const uint64_t k = count - done < 1024 ? count - done : 1024;
        for (uint64_t j = 0; j < k; j++) {
            const uint64_t i = done + j;
            const uint64_t off = offsets ? offsets[i] : i * (uint64_t)stride;
            const uint64_t len = lengths ? lengths[i] : (offsets ? offsets[i + 1] - off : stride);
            iov[j] = {const_cast<uint8_t*>(data) + off, (size_t)len};
            msgs[j] = {};
            msgs[j].msg_hdr.msg_iov = &iov[j];
            msgs[j].msg_hdr.msg_iovlen = 1;
            msgs[j].msg_hdr.msg_name = &tx->addr;
            msgs[j].msg_hdr.msg_namelen = sizeof(tx->addr);
        }
        const int r = sendmmsg(tx->fd, msgs.data(), (unsigned)k, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            if (errno == EAGAIN || errno == ENOBUFS) {  // as RawSender::send: wait for POLLOUT
                pollfd p{tx->fd, POLLOUT, 0};
                if (poll(&p, 1, 1000) <= 0) break;
                continue;
            }
            *n_sent = done;
            return NEXG_EIO;
        }
        done += (uint64_t)r;
    }
    *n_sent = done;
    return NEXG_OK;
}

int nexg_tx_close(nexg_tx* tx) {
    if (!tx) return NEXG_EINVAL;
    if (tx->fd >= 0) close(tx->fd);
    delete tx;
    return NEXG_OK;
}

}  // extern "C"
