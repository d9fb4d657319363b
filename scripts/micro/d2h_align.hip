// Which D2H copies does the runtime run as a shader blit (__amd_rocclr_copyBuffer) rather than
// on a copy engine?  Variants of one 100 MB hipMemcpyAsync into page-locked memory: aligned,
// 4-B-aligned offsets, odd sizes, several queued.  Run under rocprofv3 --kernel-trace: a blit
// shows up as a kernel between the markers (k_mark launches with the variant's id).
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/d2h_align.hip -o scripts/micro/d2h_align
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("%s: %s\n", #x, hipGetErrorString(e));                        \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void k_mark(int id, int* out) {
  if (threadIdx.x == 0 && id < 0) out[0] = id;
}

int main() {
  const size_t n = 100ull << 20;
  char *d, *h;
  int* o;
  CK(hipMalloc(&d, n + 4096));
  CK(hipMalloc(&o, 4));
  CK(hipHostMalloc((void**)&h, n + 4096, hipHostMallocPortable));
  CK(hipMemset(d, 0x5a, n + 4096));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct V {
    const char* name;
    size_t off_d, off_h, size;
    int reps;
  } vs[] = {{"aligned", 0, 0, n, 1},         {"off4 both", 4, 4, n, 1},     {"off4 dst only", 0, 4, n, 1},
            {"off4 src only", 4, 0, n, 1},   {"size+4", 0, 0, n + 4, 1},    {"off256", 256, 256, n, 1},
            {"off64", 64, 64, n, 1},         {"off16", 16, 16, n, 1},       {"4 queued aligned", 0, 0, n / 4, 4},
            {"small 64KB", 0, 0, 65536, 1},  {"small 1MB", 0, 0, 1 << 20, 1}, {"small 1MB off4", 4, 4, 1 << 20, 1}};
  int id = 0;
  for (auto& v : vs) {
    for (int w = 0; w < 2; ++w) {
      hipLaunchKernelGGL(k_mark, dim3(1), dim3(64), 0, s, id, o);
      CK(hipEventRecord(a, s));
      for (int r = 0; r < v.reps; ++r)
        CK(hipMemcpyAsync(h + v.off_h + r * v.size, d + v.off_d + r * v.size, v.size, hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(b, s));
      CK(hipStreamSynchronize(s));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (w) printf("%2d %-18s %9.3f ms %6.1f GB/s\n", id, v.name, ms, v.reps * v.size / ms / 1e6);
    }
    ++id;
  }
  return 0;
}
