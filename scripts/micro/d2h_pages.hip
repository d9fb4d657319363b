// Is the D2H rate into page-locked memory a property of the buffer's pages?  Per process,
// allocates 4 buffers of 256 MB of each kind and times 5 x 256 MB device -> mapped page-locked
// copies (kind DeviceToDeviceNoCU, as el_stream_result) into each:
//   malloc  hipHostMalloc(Portable | Mapped), as el_host_alloc did
//   thp     2-MB aligned anonymous memory with MADV_HUGEPAGE, touched, then hipHostRegister
//   4k      the same with MADV_NOHUGEPAGE
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/d2h_pages.hip -o scripts/micro/d2h_pages
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e));         \
      exit(1);                                              \
    }                                                       \
  } while (0)

static void* reg_alloc(size_t n, int advice) {
  const size_t huge = 2ull << 20;
  void* p = mmap(nullptr, n + huge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) exit(2);
  char* a = (char*)(((uintptr_t)p + huge - 1) & ~(uintptr_t)(huge - 1));
  madvise(a, n, advice);
  memset(a, 0, n);
  CK(hipHostRegister(a, n, hipHostRegisterMapped | hipHostRegisterPortable));
  return a;
}

static long anon_huge_kb() {
  FILE* f = fopen("/proc/self/smaps_rollup", "r");
  char line[256];
  long kb = -1;
  while (f && fgets(line, sizeof line, f))
    if (sscanf(line, "AnonHugePages: %ld kB", &kb) == 1) break;
  if (f) fclose(f);
  return kb;
}

int main() {
  const size_t cb = 256ull << 20;
  void* d;
  CK(hipMalloc(&d, cb));
  CK(hipMemset(d, 0x5a, cb));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* kinds[] = {"malloc", "thp", "4k"};
  for (int k = 0; k < 3; ++k)
    for (int b = 0; b < 4; ++b) {
      void* h = nullptr;
      if (k == 0)
        CK(hipHostMalloc(&h, cb, hipHostMallocPortable | hipHostMallocMapped));
      else
        h = reg_alloc(cb, k == 1 ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
      hipPointerAttribute_t at{};
      CK(hipPointerGetAttributes(&at, h));
      void* hd = at.devicePointer;
      CK(hipMemcpyAsync(hd, d, cb, hipMemcpyDeviceToDeviceNoCU, s));  // (first touch of the mapping)
      CK(hipStreamSynchronize(s));
      const auto t0 = std::chrono::steady_clock::now();
      for (int r = 0; r < 5; ++r) CK(hipMemcpyAsync(hd, d, cb, hipMemcpyDeviceToDeviceNoCU, s));
      CK(hipStreamSynchronize(s));
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      printf("%-6s buffer %d: %6.1f GB/s  (process AnonHugePages %ld kB)\n", kinds[k], b, 5 * cb / ms / 1e6,
             anon_huge_kb());
      fflush(stdout);
    }
  return 0;
}
