// Host-side checks of the index math every persistent kernel relies on (csrc/persist_common.h),
// built with the host half under AddressSanitizer + UndefinedBehaviorSanitizer
// (tests/test_native_host.py: hipcc -Xarch_host -fsanitize=...).  An out-of-range or colliding
// index here would be an out-of-bounds or racing access on the GPU, where no sanitizer runs.
//   1. frag_index is a bijection of [B, K] onto [0, B*K) (ring slabs are exactly B*K elements);
//   2. a consumer lane's frag_load_off addresses exactly the 8 elements frag_index assigns to
//      its (batch row, k-chunk) of that k-step -- producer and consumer agree on the layout;
//   3. map_block is a bijection of block ids onto (unit block, batch group) pairs, with and
//      without the XCD grouping branch.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "persist_common.h"

static int failures = 0;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      std::fprintf(stderr, __VA_ARGS__); \
      std::fprintf(stderr, "\n");       \
      if (++failures > 20) std::exit(1); \
    }                                   \
  } while (0)

static void check_frag(int B, int K) {
  const size_t n = (size_t)B * K;
  std::vector<unsigned char> seen(n, 0);
  for (int b = 0; b < B; ++b)
    for (int k = 0; k < K; ++k) {
      const size_t i = dcr::frag_index(b, k, K);
      CHECK(i < n, "frag_index(%d,%d,%d)=%zu out of [0,%zu)", b, k, K, i, n);
      if (i < n) {
        CHECK(!seen[i], "frag_index collision at %zu (b=%d k=%d K=%d)", i, b, k, K);
        seen[i] = 1;
      }
    }
  // consumer view: batch tile bt, k-step s, lane l -> row 16 bt + (l & 15), k 32 s + 8 (l >> 4)
  for (int bt = 0; bt < B / 16; ++bt)
    for (int s = 0; s < K / 32; ++s)
      for (int l = 0; l < 64; ++l) {
        const size_t want = dcr::frag_index(16 * bt + (l & 15), 32 * s + 8 * (l >> 4), K);
        const size_t got = dcr::frag_load_off(bt, s, K, l) / sizeof(dcr::bf16);
        CHECK(got == want, "frag_load_off(%d,%d,%d,%d)=%zu, frag_index says %zu", bt, s, K, l,
              got, want);
        for (int j = 1; j < 8; ++j)
          CHECK(dcr::frag_index(16 * bt + (l & 15), 32 * s + 8 * (l >> 4) + j, K) == want + j,
                "k-chunk not contiguous at bt=%d s=%d l=%d j=%d", bt, s, l, j);
      }
}

static void check_map(int nwg_u, int nbg) {
  std::vector<unsigned char> seen((size_t)nwg_u * nbg, 0);
  for (int bid = 0; bid < nwg_u * nbg; ++bid) {
    int ubk = -1, bg = -1;
    dcr::map_block(bid, nwg_u, nbg, ubk, bg);
    CHECK(ubk >= 0 && ubk < nwg_u && bg >= 0 && bg < nbg, "map_block(%d,%d,%d) -> (%d,%d)", bid,
          nwg_u, nbg, ubk, bg);
    if (ubk >= 0 && ubk < nwg_u && bg >= 0 && bg < nbg) {
      const size_t i = (size_t)bg * nwg_u + ubk;
      CHECK(!seen[i], "map_block collision (%d,%d) from bid %d", ubk, bg, bid);
      seen[i] = 1;
    }
  }
}

// map_block_grid: with the XCD-padded grid every real (unit block, column) pair is hit exactly
// once, padding blocks report false, and each column's blocks share bid % 8 (one XCD under
// round-robin dispatch); with the plain grid it is the plain column-major bijection
static void check_map_grid(int nwg_u, int ncol) {
  for (int padded = 0; padded < 2; ++padded) {
    const int grid = padded ? dcr::xcd_grid(nwg_u, ncol) : nwg_u * ncol;
    std::vector<unsigned char> seen((size_t)nwg_u * ncol, 0);
    std::vector<int> xcd(ncol, -1);
    int real = 0;
    for (int bid = 0; bid < grid; ++bid) {
      int ubk = -1, col = -1;
      if (!dcr::map_block_grid(bid, grid, nwg_u, ncol, ubk, col)) continue;
      ++real;
      CHECK(ubk >= 0 && ubk < nwg_u && col >= 0 && col < ncol, "map_block_grid(%d,%d,%d,%d)",
            bid, grid, nwg_u, ncol);
      if (ubk < 0 || ubk >= nwg_u || col < 0 || col >= ncol) continue;
      const size_t i = (size_t)col * nwg_u + ubk;
      CHECK(!seen[i], "map_block_grid collision (%d,%d) from bid %d", ubk, col, bid);
      seen[i] = 1;
      if (grid == dcr::xcd_grid(nwg_u, ncol)) {
        CHECK(xcd[col] < 0 || xcd[col] == bid % 8, "column %d spans XCD groups", col);
        xcd[col] = bid % 8;
      }
    }
    CHECK(real == nwg_u * ncol, "map_block_grid: %d real blocks, want %d", real, nwg_u * ncol);
  }
}

int main() {
  const int Bs[] = {16, 32, 48, 256};
  const int Ks[] = {32, 128, 512, 2048, 3 * 1024};
  for (int B : Bs)
    for (int K : Ks) check_frag(B, K);
  const int us[] = {1, 4, 8, 32, 64, 128};
  const int gs[] = {1, 2, 3, 8, 16, 24};
  for (int u : us)
    for (int g : gs) {
      check_map(u, g);
      check_map_grid(u, g);
    }
  if (failures) {
    std::fprintf(stderr, "%d layout check(s) failed\n", failures);
    return 1;
  }
  std::printf("layout checks ok\n");
  return 0;
}
