// Host-only stress test of the input-pipeline core (loader_core.h), built plain, under
// ASan+UBSan and under TSan (cloud_amd._build.build_loader_test, tests/test_native_sanitizers.py,
// CI).  It drives the worker pool the way the Python DeviceLoader does -- start_epoch /
// next / release from the consumer thread while the workers fill slots -- and checks:
//   * every epoch, each rank's batches are exactly its rank-strided share of one
//     permutation (no sample lost or duplicated, the ranks' shares disjoint);
//   * batches come out in order and carry the right sample count (short last batch);
//   * destroying a loader with work in flight and slots still held is clean.
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <set>

#include "loader_core.h"

using ca_data::Loader;

static int failures = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

// .npy v1.0 file of n int32 samples of `cols` values: sample i holds i in every value
static std::string write_npy(const char* dir, long n, int cols) {
  std::string path = std::string(dir) + "/samples.npy";
  char hdr[128];
  int len = snprintf(hdr, sizeof hdr, "{'descr': '<i4', 'fortran_order': False, 'shape': (%ld, %d), }", n, cols);
  int total = 10 + len + 1;
  int pad = (64 - total % 64) % 64;
  FILE* f = fopen(path.c_str(), "wb");
  fwrite("\x93NUMPY\x01\x00", 1, 8, f);
  unsigned short hl = (unsigned short)(len + pad + 1);
  fwrite(&hl, 2, 1, f);
  fwrite(hdr, 1, len, f);
  for (int i = 0; i < pad; ++i) fputc(' ', f);
  fputc('\n', f);
  std::vector<int32_t> row(cols);
  for (long i = 0; i < n; ++i) {
    for (int c = 0; c < cols; ++c) row[c] = (int32_t)i;
    fwrite(row.data(), 4, cols, f);
  }
  fclose(f);
  return path;
}

int main() {
  char dir[] = "/tmp/ca_loader_testXXXXXX";
  if (!mkdtemp(dir)) return 2;
  const long n = 1003;
  const int cols = 5, world = 3, batch = 16, nslots = 4, threads = 6;
  const std::string path = write_npy(dir, n, cols);
  for (int epoch_mode = 0; epoch_mode < 2; ++epoch_mode) {
    const bool shuffle = epoch_mode == 1;
    std::set<long> seen_all[3];
    for (int epoch = 0; epoch < 3; ++epoch) {
      std::set<long> union_epoch;
      for (int rank = 0; rank < world; ++rank) {
        std::vector<std::vector<int32_t>> bufs(nslots, std::vector<int32_t>((size_t)batch * cols));
        std::vector<std::vector<uint64_t>> slots(nslots);
        for (int s = 0; s < nslots; ++s) slots[s] = {(uint64_t)(uintptr_t)bufs[s].data()};
        Loader L({path}, batch, shuffle, 42, rank, world, false, threads, slots);
        const long nb = L.start_epoch(epoch);
        const long per = n / world;
        CHECK(nb == (per + batch - 1) / batch);
        long got = 0, order = 0;
        for (;;) {
          auto r = L.next();
          if (r.first < 0) break;
          CHECK(r.second == std::min<long>(batch, per - order * batch));
          const int32_t* b = bufs[r.first].data();
          for (long i = 0; i < r.second; ++i) {
            const int32_t v = b[i * cols];
            for (int c = 1; c < cols; ++c) CHECK(b[i * cols + c] == v);
            CHECK(v >= 0 && v < n);
            CHECK(union_epoch.insert(v).second);  // disjoint across ranks, no duplicate
          }
          got += r.second;
          ++order;
          if (order % 3 == 0) usleep(200);  // let the workers run ahead into every slot
          L.release(r.first);
        }
        CHECK(got == per);
        CHECK(order == nb);
      }
      CHECK((long)union_epoch.size() == (n / world) * world);
    }
  }
  // tear-down with batches in flight and a slot still held
  {
    std::vector<std::vector<int32_t>> bufs(nslots, std::vector<int32_t>((size_t)batch * cols));
    std::vector<std::vector<uint64_t>> slots(nslots);
    for (int s = 0; s < nslots; ++s) slots[s] = {(uint64_t)(uintptr_t)bufs[s].data()};
    Loader L({path}, batch, true, 7, 0, 1, true, threads, slots);
    L.start_epoch(0);
    auto r = L.next();
    CHECK(r.first >= 0 && r.second == batch);
    L.start_epoch(1);  // re-arm while work is pending: must wait for the in-flight fills
    auto r2 = L.next();
    CHECK(r2.first >= 0);
  }
  unlink(path.c_str());
  rmdir(dir);
  if (failures) {
    fprintf(stderr, "loader_test: %d failure(s)\n", failures);
    return 1;
  }
  printf("loader_test: ok\n");
  return 0;
}
