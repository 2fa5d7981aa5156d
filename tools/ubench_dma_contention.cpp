// Why does the reference-gather MSM path (sv_bn254_g1_msm_refs) see ~33 GB/s host->device DMA from
// its pinned staging while the contiguous path's pageable copies run at ~52 GB/s?  Measures 96 MB
// H2D copies (pinned hipHostMalloc, pageable) alone and while T host threads run a random 64-B
// gather (the library's host-pool gather) or a streaming memcpy, and reports the NUMA nodes of the
// GPU, the pinned buffer and the calling thread.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_dma_contention.cpp -o tools/ubench_dma_contention -lpthread
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static int node_of(const void* p) {  // get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR)
  int node = -1;
  if (syscall(SYS_get_mempolicy, &node, nullptr, 0, p, 3) != 0) return -1;
  return node;
}

static std::string read_file(const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return "?";
  char buf[256] = {0};
  size_t k = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  while (k && (buf[k - 1] == '\n' || buf[k - 1] == ' ')) buf[--k] = 0;
  return buf;
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)(argc > 1 ? atoi(argv[1]) : 96) << 20;
  const int T = argc > 2 ? atoi(argv[2]) : 16;
  char bus[64] = {0};
  CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
  for (char* c = bus; *c; c++) *c = (char)tolower(*c);
  cpu_set_t cs;
  sched_getaffinity(0, sizeof cs, &cs);
  printf("gpu %s numa_node %s; affinity cpus %d; hardware_concurrency %u; this thread on cpu %d node %s\n", bus,
         read_file(std::string("/sys/bus/pci/devices/") + bus + "/numa_node").c_str(), CPU_COUNT(&cs),
         std::thread::hardware_concurrency(), sched_getcpu(),
         read_file("/sys/devices/system/cpu/cpu" + std::to_string(sched_getcpu()) + "/topology/physical_package_id")
             .c_str());

  void* dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  char* pin = nullptr;
  CK(hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault));
  memset(pin, 1, bytes);
  char* page = (char*)malloc(bytes);
  memset(page, 2, bytes);
  printf("pinned buffer node %d, pageable buffer node %d\n", node_of(pin), node_of(page));

  // contention sources
  const size_t pool = size_t(1) << 30;
  char* big = (char*)malloc(pool);
  memset(big, 3, pool);
  std::atomic<int> stop{0};
  std::atomic<long> moved{0};
  auto gather = [&](int k) {
    std::mt19937_64 rng(k);
    std::vector<char> out(8 << 20);
    size_t o = 0;
    long m = 0;
    while (!stop.load(std::memory_order_relaxed)) {
      for (int r = 0; r < 1024; r++) {
        const size_t at = (rng() % (pool / 64)) * 64;
        memcpy(&out[o], big + at, 64);
        o = (o + 64) % out.size();
      }
      m += 1024 * 64;
    }
    moved += m;
  };
  auto stream = [&](int k) {
    std::vector<char> out(64 << 20);
    const size_t span = pool / T, lo = (size_t)k * span;
    long m = 0;
    size_t o = 0;
    while (!stop.load(std::memory_order_relaxed)) {
      const size_t len = std::min(out.size(), span);
      memcpy(out.data(), big + lo + (o % (span - len + 1)), len);
      o += len;
      m += (long)len;
    }
    moved += m;
  };

  auto time_copy = [&](const char* what, const void* src, int load, int threads) {
    std::vector<std::thread> th;
    stop = 0;
    moved = 0;
    for (int k = 0; k < (load ? threads : 0); k++) th.emplace_back(load == 1 ? std::function<void()>([&, k] { gather(k); })
                                                                         : std::function<void()>([&, k] { stream(k); }));
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    CK(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    const int reps = 5;
    const double t0 = now_ms();
    for (int r = 0; r < reps; r++) CK(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    const double ms = (now_ms() - t0) / reps;
    const double wall = now_ms() - t0 + 20;
    stop = 1;
    for (auto& t : th) t.join();
    printf("%-10s %-22s %8.3f ms %7.1f GB/s   (host load moved %.1f GB/s)\n", what,
           load == 0 ? "alone" : (load == 1 ? "+ random gather" : "+ streaming memcpy"), ms, bytes / ms / 1e6,
           moved.load() / wall / 1e6);
  };
  for (int load : {0, 1, 2}) {
    time_copy("pinned", pin, load, T);
    time_copy("pageable", page, load, T);
  }
  for (int t2 : {4, 8}) {
    printf("-- %d gather threads\n", t2);
    time_copy("pinned", pin, 1, t2);
    time_copy("pageable", page, 1, t2);
  }
  return 0;
}
