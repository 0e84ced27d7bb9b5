// TEST INFRASTRUCTURE ONLY: drives nex_amd/csrc/nexg_pcap.cpp (built here
// with AddressSanitizer + UBSan) over every file named on the command line,
// through both batch shapes and small buffers, so malformed captures are
// exercised for memory safety. Exit 0 = no crash / sanitizer report.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/nexg.h"

static void drain(const char* path, bool raw, uint64_t cap, uint64_t maxf) {
    nexg_pcap* p = nullptr;
    if (nexg_pcap_open(path, &p) != NEXG_OK) return;
    std::vector<uint8_t> buf(cap);
    std::vector<uint64_t> offs(maxf + 1);
    std::vector<uint32_t> lens(maxf);
    std::vector<uint64_t> ts(maxf);
    for (int guard = 0; guard < 100000; guard++) {
        uint64_t n = 0, used = 0;
        int rc = raw ? nexg_pcap_read_raw(p, buf.data(), cap, offs.data(), lens.data(), maxf, ts.data(), &n, &used)
                     : nexg_pcap_read_batch(p, buf.data(), cap, offs.data(), maxf, ts.data(), &n);
        if (rc != NEXG_OK) break;
        for (uint64_t k = 0; k < n; k++) {  // every delivered frame lies inside buf
            const uint64_t a = raw ? offs[k] : offs[k], l = raw ? lens[k] : offs[k + 1] - offs[k];
            if (a + l > cap) { fprintf(stderr, "frame outside buffer\n"); abort(); }
            volatile uint8_t x = l ? buf[a + l - 1] : 0;
            (void)x;
        }
        if (n == 0 && (!raw || used == 0)) break;
    }
    nexg_pcap_close(p);
}

int main(int argc, char** argv) {
    for (int i = 1; i < argc; i++) {
        drain(argv[i], false, 1 << 20, 64);
        drain(argv[i], false, 2000, 3);
        drain(argv[i], true, 1 << 20, 64);
        drain(argv[i], true, 3000, 5);
    }
    return 0;
}
