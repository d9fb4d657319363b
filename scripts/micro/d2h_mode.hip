// Which D2H copies into page-locked memory does the HIP runtime run as blit kernels (CUs) and
// which on an SDMA engine?  Each case copies 64 MB device -> page-locked host memory 20 times on
// stream s1 while a bandwidth-bound kernel runs on s0, the way el_stream_result does.  Run under
// `rocprofv3 --kernel-trace`: a case whose copies appear as __amd_rocclr_copyBuffer kernels ran as
// blits.  Cases (printed with their time stamps so the trace can be split):
//   A  dst = the mapped device address of the buffer, kind DeviceToDeviceNoCU   (the engine's)
//   B  dst = the host pointer, kind DeviceToHost
//   C  B behind an event (hipEventReleaseToSystem) recorded on s0 after a kernel
//   D  A behind that event
//   E  dst = host pointer, kind Default
// (argv[1]: run only the case with that letter, so each case can get a trace of its own)
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/d2h_mode.hip -o scripts/micro/d2h_mode
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      exit(1);                                                      \
    }                                                               \
  } while (0)

__global__ void k_read(const uint4* __restrict__ a, size_t n, unsigned* out) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

int main(int argc, char** argv) {
  const char only = argc > 1 ? argv[1][0] : 0;  // one case (its letter), or all
  const size_t cb = 64ull << 20, kb = 2ull << 30;
  void *d, *big, *h;
  unsigned* o;
  CK(hipMalloc(&d, cb));
  CK(hipMalloc(&big, kb));
  CK(hipMalloc(&o, 4));
  CK(hipHostMalloc(&h, cb, hipHostMallocPortable));
  CK(hipMemset(d, 0x5a, cb));
  CK(hipMemset(big, 1, kb));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, h));
  void* hd = at.devicePointer;
  printf("host %p device view %p (%s)\n", h, hd, h == hd ? "same address" : "different address");
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToSystem));
  struct Case {
    const char* name;
    bool dev_dst, after_event;
    hipMemcpyKind kind;
  } cases[] = {{"A dev-dst D2D-NoCU", true, false, hipMemcpyDeviceToDeviceNoCU},
               {"B host-dst D2H", false, false, hipMemcpyDeviceToHost},
               {"C host-dst D2H after event", false, true, hipMemcpyDeviceToHost},
               {"D dev-dst D2D-NoCU after event", true, true, hipMemcpyDeviceToDeviceNoCU},
               {"E host-dst Default", false, false, hipMemcpyDefault}};
  for (auto& c : cases) {
    if (only && c.name[0] != only) continue;
    CK(hipDeviceSynchronize());
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < 20; ++r) {
      hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, s0, (const uint4*)big, kb / 16, o);
      if (c.after_event) {
        CK(hipEventRecord(ev, s0));
        CK(hipStreamWaitEvent(s1, ev, 0));
      }
      CK(hipMemcpyAsync(c.dev_dst ? hd : h, d, cb, c.kind, s1));
    }
    CK(hipDeviceSynchronize());
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    printf("%-32s %8.3f ms for 20 x (kernel + 64 MB copy)\n", c.name, ms);
    fflush(stdout);
  }
  return 0;
}
