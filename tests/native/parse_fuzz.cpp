// TEST INFRASTRUCTURE ONLY: the device parse core (frame_core.hpp, through
// core_harness.hip's host accessors) and the oracle, both built with
// AddressSanitizer + UBSan, over every frame of the input file (records of
// u32 length + bytes). Each frame sits alone in a heap block that ends at the
// frame's last 16-B chunk (the kernels' load granule), at three alignments, in
// six parse modes, through four window/fast-path variants: any read outside
// the frame's chunks is a sanitizer report, any record / FrameSlice that
// differs from the oracle's is counted. The analogue of the reference's
// panic_free_parsing.rs. Exit 0 = clean and equal.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/nexg.h"
#include "../../oracle/nex_oracle.h"

extern "C" int harness_parse(const uint8_t* data, uint64_t data_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t stride, uint64_t count, uint32_t flags,
                             uint32_t ip_offset, uint32_t window, int use_fast, nexg_record* out);
extern "C" int harness_slice(const uint8_t* data, uint64_t data_bytes, const uint64_t* offsets,
                             const uint32_t* lengths, uint32_t stride, uint64_t count, uint32_t flags,
                             uint32_t ip_offset, uint32_t window, nexg_slice* out);

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<std::vector<uint8_t>> frames;
    uint32_t len;
    while (fread(&len, 4, 1, f) == 1) {
        std::vector<uint8_t> b(len);
        if (len && fread(b.data(), 1, len, f) != len) return 2;
        frames.push_back(std::move(b));
    }
    fclose(f);
    const uint32_t modes[][2] = {{0, 0}, {NEXG_PARSE_STRICT, 0}, {NEXG_PARSE_FROM_IP, 0},
                                 {NEXG_PARSE_FROM_IP, 14}, {NEXG_PARSE_FROM_IP | NEXG_PARSE_STRICT, 14},
                                 {NEXG_PARSE_VLAN, 0}};
    const int variants[][2] = {{64, 0}, {128, 1}, {80, 4}, {128, 5}};
    long bad = 0, runs = 0;
    for (const auto& fr : frames) {
        for (uint32_t o : {0u, 3u, 14u}) {
            const size_t cap = (o + fr.size() + 15u) & ~(size_t)15u;
            uint8_t* buf = static_cast<uint8_t*>(aligned_alloc(16, cap ? cap : 16));
            memset(buf, 0x5A, cap ? cap : 16);
            if (!fr.empty()) memcpy(buf + o, fr.data(), fr.size());
            const uint8_t* g = buf + o;
            const uint64_t off0 = 0;
            const uint32_t l = (uint32_t)fr.size();
            for (const auto& m : modes) {
                nexg_record want, got;
                nexo_parse_frame(g, l, m[0], m[1], &want);
                for (const auto& v : variants) {
                    harness_parse(g, l, &off0, &l, 0, 1, m[0], m[1], (uint32_t)v[0], v[1], &got);
                    runs++;
                    if (memcmp(&want, &got, sizeof(want)) != 0 && bad++ < 5)
                        fprintf(stderr, "record differs: len %u flags %u window %d fast %d\n", l, m[0], v[0], v[1]);
                }
                nexg_slice sw, sg;
                nexo_slice_frame(g, l, m[0], m[1], &sw);
                harness_slice(g, l, &off0, &l, 0, 1, m[0], m[1], 128, &sg);
                if (memcmp(&sw, &sg, sizeof(sw)) != 0 && bad++ < 5)
                    fprintf(stderr, "slice differs: len %u flags %u\n", l, m[0]);
                nexg_options opts;
                nexo_decode_options(g, l, m[0], m[1], &opts);
            }
            free(buf);
        }
    }
    printf("frames %zu runs %ld mismatches %ld\n", frames.size(), runs, bad);
    return bad ? 1 : 0;
}
