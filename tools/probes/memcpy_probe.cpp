// Experiments only: host copy rates the streaming receiver's chunk dispatch depends on
// (2 KB rows from a hipHostMalloc buffer / from ordinary memory into a populated arena,
// 1 and 8 threads). Build: hipcc -O2 -o memcpy_probe memcpy_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
int main() {
  const size_t n = 32000, row = 2272, len = 2048, bytes = n * row;
  void *pin = nullptr;
  if (hipHostMalloc(&pin, bytes, hipHostMallocDefault) != hipSuccess) return 1;
  std::vector<uint8_t> mem(bytes, 1);
  memset(pin, 1, bytes);
  uint8_t *dst = (uint8_t *)mmap(nullptr, n * len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  madvise(dst, n * len, 23 /* MADV_POPULATE_WRITE */);
  auto run = [&](const uint8_t *src, int nt) {
    const double t0 = now_ms();
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (size_t i = t; i < n; i += nt) memcpy(dst + i * len, src + i * row, len);
      });
    for (auto &x : th) x.join();
    return now_ms() - t0;
  };
  for (int rep = 0; rep < 2; ++rep)
    for (int nt : {1, 8})
      printf("threads %d: from pinned %.3f ms, from pageable %.3f ms (%.1f MB)\n", nt,
             run((const uint8_t *)pin, nt), run(mem.data(), nt), n * len / 1e6);
  uint8_t *fresh = (uint8_t *)mmap(nullptr, n * len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  const double t0 = now_ms();
  for (size_t i = 0; i < n; ++i) memcpy(fresh + i * len, mem.data() + i * row, len);
  printf("into a fresh (unpopulated) mapping, 1 thread: %.3f ms\n", now_ms() - t0);
  return 0;
}
