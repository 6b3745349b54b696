// run_jellyfish — drop-in for src/occurrences/run_jellyfish.sh (`<reads> <k> <sorted_path>`):
// `jellyfish bc/count -C --bc` + `dump -c` + `LC_ALL=C sort` (run_jellyfish.sh:3-6) on the GPU.
// Writes the "<KMER> <count>" dump of canonical k-mers with count >= 2, ascending, to
// <sorted_path>.  bin/run_jellyfish.sh wraps it under the reference's script name, so the
// reference's popen (JellyfishOccurrenceReader.cpp:21-22) can be pointed at it unchanged.
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "hga.h"
#include "seqio.h"

int main(int argc, char* argv[]) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s <reads> <k> <sorted_path>\n", argv[0]);
        return 2;
    }
    const std::string reads = argv[1], out = argv[3];
    const int k = std::atoi(argv[2]);
    const char* dev_env = std::getenv("HGA_DEVICE");
    hga_ctx* ctx = nullptr;
    auto check = [](hga_status s, const char* what) {
        if (s != HGA_OK) throw std::runtime_error(std::string(what) + ": " + hga_last_error());
    };
    check(hga_ctx_create(&ctx, dev_env ? std::atoi(dev_env) : 0), "hga_ctx_create");
    check(hga_count_begin(ctx, k, 1), "hga_count_begin");
    const hgah::Bytes s = hgah::jf_stream(reads);
    check(hga_count_add(ctx, 0, s.data(), s.size()), "hga_count_add");
    check(hga_count_run(ctx, 2), "hga_count_run");
    uint64_t *keys = nullptr, n = 0;
    uint32_t* counts = nullptr;
    check(hga_count_dump(ctx, 0, &keys, &counts, &n), "hga_count_dump");
    hgah::write_kmer_dump(out, k, keys, counts, n);
    hga_free(keys);
    hga_free(counts);
    hga_ctx_destroy(ctx);
    return 0;
}
