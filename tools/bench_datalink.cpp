// bench_datalink.cpp — live AF_PACKET rate over loopback: the reference's
// per-frame channel pattern (poll + sendto per frame, nex-datalink/src/
// linux.rs:302-346; poll + recvfrom into a 4096-B buffer per frame,
// linux.rs:356-397) against the batch rx/tx of include/nexg.h (sendmmsg;
// TPACKET_V3 ring or recvmmsg into packed batches). Host-only, needs
// CAP_NET_RAW; one JSON line per tx mode and per rx mode on stdout.
//
// usage: bench_datalink [frames] [frame_bytes]   (defaults 200000, 64)
#include <arpa/inet.h>
#include <errno.h>
#include <linux/if_packet.h>
#include <net/ethernet.h>
#include <net/if.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <thread>
#include <vector>

#include "../include/nexg.h"

static double now_s() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static const uint8_t kTag[6] = {0x02, 0x6E, 0x65, 0x78, 0x42, 0x00};

// Eth/IPv4/UDP frames of `len` bytes from a test source MAC (so other loopback
// traffic is not counted), a sequence number in the UDP payload
static std::vector<uint8_t> make_frames(uint64_t n, uint32_t len) {
    std::vector<uint8_t> d(n * len, 0);
    for (uint64_t i = 0; i < n; i++) {
        uint8_t* f = d.data() + i * len;
        memset(f, 0xFF, 6);
        memcpy(f + 6, kTag, 6);
        f[12] = 0x08;
        f[14] = 0x45;
        const uint32_t tot = len - 14;
        f[16] = (uint8_t)(tot >> 8);
        f[17] = (uint8_t)tot;
        f[22] = 64;
        f[23] = 17;
        memcpy(f + 42, &i, 8);
    }
    return d;
}

static bool tagged(const uint8_t* f, uint32_t len) { return len >= 12 && memcmp(f + 6, kTag, 6) == 0; }

static int raw_socket(const char* ifname, sockaddr_ll* a) {
    const int fd = socket(AF_PACKET, SOCK_RAW, htons(ETH_P_ALL));
    if (fd < 0) return -1;
    memset(a, 0, sizeof(*a));
    a->sll_family = AF_PACKET;
    a->sll_protocol = htons(ETH_P_ALL);
    a->sll_ifindex = (int)if_nametoindex(ifname);
    if (bind(fd, reinterpret_cast<sockaddr*>(a), sizeof(*a)) < 0) {
        close(fd);
        return -1;
    }
    return fd;
}

// the reference's RawSender::send: poll(POLLOUT) + sendto, one frame per call
static uint64_t send_per_frame(const std::vector<uint8_t>& d, uint64_t n, uint32_t len) {
    sockaddr_ll a;
    const int fd = raw_socket("lo", &a);
    if (fd < 0) return 0;
    uint64_t sent = 0;
    for (uint64_t i = 0; i < n; i++) {
        pollfd p{fd, POLLOUT, 0};
        if (poll(&p, 1, 1000) <= 0) break;
        if (sendto(fd, d.data() + i * len, len, 0, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == (ssize_t)len) sent++;
    }
    close(fd);
    return sent;
}

static uint64_t send_batch(const std::vector<uint8_t>& d, uint64_t n, uint32_t len) {
    nexg_tx* tx = nullptr;
    if (nexg_tx_open("lo", &tx)) return 0;
    uint64_t sent = 0, done = 0;
    while (done < n) {  // 4096-frame calls, as a ring of pinned batches would hand them over
        const uint64_t k = n - done < 4096 ? n - done : 4096;
        uint64_t s = 0;
        if (nexg_tx_send_batch(tx, d.data() + done * len, nullptr, nullptr, len, k, &s)) break;
        sent += s;
        done += k;
    }
    nexg_tx_close(tx);
    return sent;
}

struct RxResult {
    uint64_t frames = 0;
    double first = 0, last = 0;
};

// the reference's RawReceiver::next: poll(POLLIN) + recvfrom into 4096 B
static void recv_per_frame(int fd, uint64_t want, std::atomic<bool>& stop, RxResult& r) {
    std::vector<uint8_t> buf(4096);
    while (r.frames < want && !stop.load()) {
        pollfd p{fd, POLLIN, 0};
        if (poll(&p, 1, 200) <= 0) continue;
        const ssize_t got = recvfrom(fd, buf.data(), buf.size(), 0, nullptr, nullptr);
        if (got > 0 && tagged(buf.data(), (uint32_t)got)) {
            if (r.frames == 0) r.first = now_s();
            r.frames++;
            r.last = now_s();
        }
    }
}

// the batch buffers are allocated (and touched) once, outside the timing, as
// a pinned staging ring would be
static const uint64_t kMaxBatch = 65536;
static std::vector<uint8_t> g_data(kMaxBatch * 2048, 1);
static std::vector<uint64_t> g_offs(kMaxBatch + 1, 0);

static void recv_batch(nexg_rx* rx, uint64_t want, std::atomic<bool>& stop, RxResult& r) {
    const uint64_t maxf = kMaxBatch;
    std::vector<uint8_t>& data = g_data;
    std::vector<uint64_t>& offs = g_offs;
    while (r.frames < want && !stop.load()) {
        uint64_t n = 0;
        if (nexg_rx_next_batch(rx, data.data(), data.size(), offs.data(), maxf, nullptr, &n)) break;
        uint64_t t = 0;
        for (uint64_t k = 0; k < n; k++) t += tagged(data.data() + offs[k], (uint32_t)(offs[k + 1] - offs[k]));
        if (t) {
            if (r.frames == 0) r.first = now_s();
            r.frames += t;
            r.last = now_s();
        }
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 200000;
    const uint32_t len = argc > 2 ? (uint32_t)strtoul(argv[2], nullptr, 10) : 64;
    const auto frames = make_frames(n, len);
    // tx: frames handed to the kernel per second, no receiver open
    for (int t = 0; t < 2; t++) {
        const double t0 = now_s();
        const uint64_t sent = t == 0 ? send_per_frame(frames, n, len) : send_batch(frames, n, len);
        const double t1 = now_s();
        printf("{\"side\": \"tx\", \"mode\": \"%s\", \"frame_bytes\": %u, \"frames\": %llu, \"mpps\": %.3f}\n",
               t == 0 ? "per_frame_poll_sendto (reference linux.rs:302-346)" : "sendmmsg_batch (nexg_tx_send_batch)", len,
               (unsigned long long)sent, sent / (t1 - t0) / 1e6);
        fflush(stdout);
    }
    // rx: the frames are queued first (loopback delivers each twice to a
    // packet socket: outgoing + host copy), then the application drains them;
    // the drain rate is what the receive API costs the application
    const char* rxs[] = {"per_frame_poll_recvfrom (reference linux.rs:356-397)", "tpacket_v3_ring (nexg_rx_next_batch)",
                         "recvmmsg (nexg_rx_next_batch)"};
    for (int m = 0; m < 3; m++) {
        std::atomic<bool> stop{false};
        RxResult r;
        int fd = -1;
        nexg_rx* rx = nullptr;
        if (m == 0) {
            sockaddr_ll a;
            fd = raw_socket("lo", &a);
            if (fd < 0) { fprintf(stderr, "AF_PACKET: %s\n", strerror(errno)); return 1; }
            const int big = 1 << 30;  // the same queue depth as the batch receivers
            if (setsockopt(fd, SOL_SOCKET, SO_RCVBUFFORCE, &big, sizeof(big)) < 0)
                (void)setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
        } else {
            nexg_rx_config c;
            nexg_rx_config_default(&c);
            c.read_timeout_ms = 200;
            c.promiscuous = 0;
            c.ring_blocks = 512;  // 512 MiB ring: a whole burst is queued before the drain
            c.mode = m == 1 ? NEXG_RX_RING : NEXG_RX_MMSG;
            if (nexg_rx_open("lo", &c, &rx)) { fprintf(stderr, "nexg_rx_open failed\n"); return 1; }
        }
        // two rounds on the same receiver, the second reported: the first
        // also pays the page faults that map the ring into the process
        uint64_t sent = 0;
        double t0 = 0, t1 = 0;
        for (int round = 0; round < 2; round++) {
            r = RxResult{};
            sent = send_batch(frames, n, len);
            usleep(200000);  // let the last ring block retire (block timeout)
            t0 = now_s();
            if (m == 0) recv_per_frame(fd, 2 * sent, stop, r);
            else recv_batch(rx, 2 * sent, stop, r);
            t1 = now_s();
        }
        uint64_t pk = 0, dr = 0;
        if (rx) {
            nexg_rx_stats(rx, &pk, &dr);
            nexg_rx_close(rx);
        }
        if (fd >= 0) close(fd);
        printf("{\"side\": \"rx\", \"mode\": \"%s\", \"frame_bytes\": %u, \"copies\": %llu, \"expected\": %llu, "
               "\"drain_mpps\": %.3f, \"kernel_drops\": %llu}\n",
               rxs[m], len, (unsigned long long)r.frames, (unsigned long long)(2 * sent), r.frames / (t1 - t0) / 1e6,
               (unsigned long long)dr);
        fflush(stdout);
    }
    // rx scale-out: K TPACKET_V3 receivers in one PACKET_FANOUT (hash) group,
    // one drain thread each (one receiver per GPU); the
    // burst's frames differ in their IPv4 source so the hash spreads them
    for (uint32_t K : {2u, 4u}) {
        auto fr = frames;
        for (uint64_t i = 0; i < n; i++) memcpy(fr.data() + i * len + 26, &i, 4);  // IPv4 source address
        std::vector<nexg_rx*> rxv(K, nullptr);
        for (uint32_t k = 0; k < K; k++) {
            nexg_rx_config c;
            nexg_rx_config_default(&c);
            c.read_timeout_ms = 200;
            c.promiscuous = 0;
            c.ring_blocks = 512;  // the hash may put most of a burst on one member
            c.fanout = 1;
            c.fanout_type = NEXG_FANOUT_HASH;
            c.fanout_group = 0x4E40u + K;
            if (nexg_rx_open("lo", &c, &rxv[k])) { fprintf(stderr, "nexg_rx_open (fanout) failed\n"); return 1; }
        }
        double best = 0;
        uint64_t got = 0, sent = 0;
        for (int round = 0; round < 2; round++) {
            sent = send_batch(fr, n, len);
            usleep(200000);
            std::vector<RxResult> rr(K);
            std::vector<std::atomic<bool>> stops(K);
            std::vector<std::vector<uint8_t>> bufs(K, std::vector<uint8_t>(kMaxBatch * 2048, 1));
            std::vector<std::vector<uint64_t>> offv(K, std::vector<uint64_t>(kMaxBatch + 1, 0));
            std::vector<std::thread> th;
            const double t0 = now_s();
            for (uint32_t k = 0; k < K; k++)
                th.emplace_back([&, k] {  // drain until the receiver's queue stays empty for a timeout
                    for (;;) {
                        uint64_t m = 0;
                        if (nexg_rx_next_batch(rxv[k], bufs[k].data(), bufs[k].size(), offv[k].data(), kMaxBatch,
                                               nullptr, &m) || m == 0)
                            break;
                        for (uint64_t j = 0; j < m; j++)
                            rr[k].frames += tagged(bufs[k].data() + offv[k][j], (uint32_t)(offv[k][j + 1] - offv[k][j]));
                        rr[k].last = now_s();
                    }
                });
            for (auto& x : th) x.join();
            got = 0;
            double last = t0;
            for (auto& x : rr) {
                got += x.frames;
                last = x.last > last ? x.last : last;
            }
            best = got / (last - t0) / 1e6;
        }
        uint64_t drops = 0;
        for (auto* x : rxv) {
            uint64_t pk = 0, dr = 0;
            nexg_rx_stats(x, &pk, &dr);
            drops += dr;
            nexg_rx_close(x);
        }
        printf("{\"side\": \"rx\", \"mode\": \"%u x tpacket_v3_ring in one PACKET_FANOUT hash group, one thread each\", "
               "\"frame_bytes\": %u, \"copies\": %llu, \"expected\": %llu, \"drain_mpps\": %.3f, \"kernel_drops\": %llu}\n",
               K, len, (unsigned long long)got, (unsigned long long)(2 * sent), best, (unsigned long long)drops);
        fflush(stdout);
    }
    return 0;
}
