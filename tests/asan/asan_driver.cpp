// Host-sanitizer driver for the native runtime's input-parsing paths: built with
// ASan + UBSan on the host code only (tests/asan/build.sh) and run by tests/test_asan_runtime.py on the
// CPU. It feeds the BSG1 weight-blob parser + BN folding + packer (bugseg_debug_parse_pack = what
// bugseg_load_weights does before the upload), the DeepLab plan validator (bugseg_dl_debug_check_plan
// = bugseg_dl_set_plan before the allocation) and the polar-table builder with valid inputs, every
// truncation of the blob's head and a sample of the rest, and seeded corruptions. Any out-of-bounds
// access, use-after-free or undefined behaviour aborts the process (exit status != 0); a rejected input
// is the expected outcome for a corrupted one.
//
// usage: asan_driver <enet.bsg1> <dl_ops.i32> <dl_bufs.u64> <B> <Hc> <Wc> <dl_w_bytes> <dl_precision>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <vector>

#include "../../include/bugseg.h"

static std::vector<unsigned char> slurp(const char *path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { std::fprintf(stderr, "cannot read %s\n", path); std::exit(2); }
    return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct Rng {   // xorshift64*, fixed seed: the run is reproducible
    uint64_t s = 0x9E3779B97F4A7C15ull;
    uint64_t next() { s ^= s >> 12; s ^= s << 25; s ^= s >> 27; return s * 2685821657736338717ull; }
    uint32_t below(uint32_t n) { return (uint32_t)(next() % n); }
};

static const uint32_t kExtreme[] = {0u, 1u, 2u, 3u, 7u, 8u, 16u, 127u, 128u, 255u, 4096u, 65535u, 0x7fffffffu, 0x80000000u, 0xffffffffu, 0xfffffff0u};

int main(int argc, char **argv) {
    if (argc != 9) { std::fprintf(stderr, "usage: %s enet.bsg1 dl_ops.i32 dl_bufs.u64 B Hc Wc w_bytes prec\n", argv[0]); return 2; }
    const std::vector<unsigned char> blob = slurp(argv[1]);
    const std::vector<unsigned char> ops_raw = slurp(argv[2]), bufs_raw = slurp(argv[3]);
    const int B = std::atoi(argv[4]), Hc = std::atoi(argv[5]), Wc = std::atoi(argv[6]), prec = std::atoi(argv[8]);
    const size_t w_bytes = (size_t)std::strtoull(argv[7], nullptr, 10);
    Rng rng;
    long accepted = 0, rejected = 0;
    auto tally = [&](int rc) { (rc == BUGSEG_OK ? accepted : rejected)++; };

    // ---- the ENet weight blob, both precisions
    for (int p = 0; p < 2; ++p) {
        int ncls = 0;
        if (bugseg_debug_parse_pack(blob.data(), blob.size(), p, &ncls) != BUGSEG_OK || ncls < 1) {
            std::fprintf(stderr, "valid blob rejected: %s\n", bugseg_last_error(nullptr));
            return 1;
        }
    }
    // truncations: every length of the first 4 KB, then a stride through the rest (each in a buffer
    // of exactly that size, so a read past the end is a heap overflow ASan reports)
    for (size_t n = 0; n < blob.size(); n += n < 4096 ? 1 : 997) {
        std::vector<unsigned char> t(blob.begin(), blob.begin() + n);
        tally(bugseg_debug_parse_pack(t.empty() ? nullptr : t.data(), t.size(), 1, nullptr));
        if (!t.empty()) tally(bugseg_debug_parse_pack(t.data(), t.size(), 0, nullptr));
    }
    // corruptions: random bytes, and 32-bit header / shape / count fields set to extreme values
    for (int it = 0; it < 3000; ++it) {
        std::vector<unsigned char> t = blob;
        const int edits = 1 + (int)rng.below(4);
        for (int e = 0; e < edits; ++e) {
            if (rng.below(2)) {
                t[rng.below((uint32_t)t.size())] = (unsigned char)rng.next();
            } else {
                // a 4-byte-aligned field in the first 64 KB (headers, unit dims, tensor lengths live there)
                const uint32_t lim = (uint32_t)std::min<size_t>(t.size(), 65536) / 4;
                const uint32_t off = rng.below(lim) * 4;
                const uint32_t v = kExtreme[rng.below(sizeof(kExtreme) / sizeof(kExtreme[0]))];
                if (off + 4 <= t.size()) std::memcpy(&t[off], &v, 4);
            }
        }
        tally(bugseg_debug_parse_pack(t.data(), t.size(), (int)rng.below(2), nullptr));
    }

    // ---- the DeepLab op list
    const int nf = BUGSEG_DL_OP_FIELDS;
    const int nops = (int)(ops_raw.size() / (4 * nf)), nbufs = (int)(bufs_raw.size() / 8);
    std::vector<int32_t> ops(ops_raw.size() / 4);
    std::memcpy(ops.data(), ops_raw.data(), ops.size() * 4);
    std::vector<uint64_t> bufs(nbufs);
    std::memcpy(bufs.data(), bufs_raw.data(), bufs.size() * 8);
    if (bugseg_dl_debug_check_plan(ops.data(), nops, bufs.data(), nbufs, B, Hc, Wc, prec, w_bytes) != BUGSEG_OK) {
        std::fprintf(stderr, "valid plan rejected: %s\n", bugseg_dl_last_error(nullptr));
        return 1;
    }
    for (int it = 0; it < 20000; ++it) {
        std::vector<int32_t> o = ops;
        std::vector<uint64_t> b = bufs;
        const int edits = 1 + (int)rng.below(3);
        for (int e = 0; e < edits; ++e) {
            const uint32_t r = rng.below(10);
            if (r < 8) {
                const uint32_t v = kExtreme[rng.below(sizeof(kExtreme) / sizeof(kExtreme[0]))];
                o[rng.below((uint32_t)o.size())] = rng.below(3) ? (int32_t)v : (int32_t)rng.next();
            } else {
                b[rng.below((uint32_t)b.size())] = rng.below(2) ? 0 : rng.next();
            }
        }
        // occasionally a shorter op list / buffer table: the count arguments must bound every access
        const int n_ops = rng.below(8) ? nops : 1 + (int)rng.below((uint32_t)nops);
        const int n_bufs = rng.below(8) ? nbufs : 1 + (int)rng.below((uint32_t)nbufs);
        std::vector<int32_t> oc(o.begin(), o.begin() + (size_t)n_ops * nf);
        std::vector<uint64_t> bc(b.begin(), b.begin() + n_bufs);
        tally(bugseg_dl_debug_check_plan(oc.data(), n_ops, bc.data(), n_bufs, B, Hc, Wc, prec,
                                         rng.below(4) ? w_bytes : (size_t)rng.below((uint32_t)w_bytes + 1)));
    }
    tally(bugseg_dl_debug_check_plan(nullptr, nops, bufs.data(), nbufs, B, Hc, Wc, prec, w_bytes));
    tally(bugseg_dl_debug_check_plan(ops.data(), 0, bufs.data(), nbufs, B, Hc, Wc, prec, w_bytes));

    // ---- polar tables (laserscan mode): small, odd, degenerate and large geometries
    const int geo[][2] = {{1, 1}, {1, 7}, {7, 1}, {2, 3}, {31, 27}, {200, 200}, {50, 120}, {300, 40}, {1000, 3}};
    for (const auto &g : geo)
        for (int variant = 0; variant < 2; ++variant) {
            int pw = 0, ph = 0;
            if (bugseg_debug_polar_tables(g[0], g[1], variant, nullptr, 0, nullptr, 0, &pw, &ph) != BUGSEG_OK) continue;
            std::vector<int32_t> fm((size_t)pw * ph), im((size_t)g[0] * g[1]);
            tally(bugseg_debug_polar_tables(g[0], g[1], variant, fm.data(), fm.size(), im.data(), im.size(), &pw, &ph));
            for (int32_t v : fm) if (v != -1 && ((v & 0xffff) >= g[0] || (v >> 16) >= g[1])) { std::fprintf(stderr, "fmap out of grid\n"); return 1; }
            for (int32_t v : im) if (v != -1 && ((v & 0xffff) >= pw || (v >> 16) >= ph)) { std::fprintf(stderr, "imap out of polar image\n"); return 1; }
        }
    tally(bugseg_debug_polar_tables(0, 5, 0, nullptr, 0, nullptr, 0, nullptr, nullptr));
    tally(bugseg_debug_polar_tables(40000, 5, 0, nullptr, 0, nullptr, 0, nullptr, nullptr));

    std::printf("asan driver ok: %ld inputs accepted, %ld rejected\n", accepted, rejected);
    return 0;
}
