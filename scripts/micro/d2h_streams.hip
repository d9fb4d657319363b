// Is the D2H rate of a stream's copies into page-locked memory a property of the stream (the
// hardware queue / SDMA engine the runtime binds it to)?  Creates streams one after another (the
// way engines created and destroyed in one process do) and times 10 x 64 MB device -> mapped
// page-locked copies (kind DeviceToDeviceNoCU, as el_stream_result) on each, alone and beside a
// bandwidth-bound kernel on a second stream.  argv[1]: streams to try (default 12);
// argv[2] = "d": destroy each stream pair before creating the next; argv[3]: where the page-locked
// buffer lives — "p" hipHostMallocPortable as el_host_alloc did (the runtime picks the pool),
// "near" / "far": the calling thread bound (affinity + MPOL_BIND) to the GPU's NUMA node or the
// other one, with hipHostMallocNumaUser so the allocation follows that policy.
// Build: hipcc --offload-arch=gfx950 -O2 scripts/micro/d2h_streams.hip -o scripts/micro/d2h_streams
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

static int gpu_node() {
  char bus[64];
  if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) != hipSuccess) return -1;
  for (char* c = bus; *c; ++c) *c = (char)tolower(*c);
  char path[256];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE* f = fopen(path, "r");
  int n = -1;
  if (f) {
    if (fscanf(f, "%d", &n) != 1) n = -1;
    fclose(f);
  }
  return n;
}

static void bind_node(int node) {  // CPUs of the node (sysfs cpulist) + MPOL_BIND to it
  char path[128], buf[4096];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f || !fgets(buf, sizeof buf, f)) exit(2);
  fclose(f);
  cpu_set_t set;
  CPU_ZERO(&set);
  for (char* t = strtok(buf, ",\n"); t; t = strtok(nullptr, ",\n")) {
    int a = 0, b = 0;
    if (sscanf(t, "%d-%d", &a, &b) != 2) b = a = atoi(t);
    for (int c = a; c <= b; ++c) CPU_SET(c, &set);
  }
  sched_setaffinity(0, sizeof set, &set);
  unsigned long mask = 1ul << node;
  syscall(SYS_set_mempolicy, 2 /* MPOL_BIND */, &mask, 8 * sizeof mask);
}

#define CK(x)                                               \
  do {                                                      \
    hipError_t e = (x);                                     \
    if (e != hipSuccess) {                                  \
      printf("%s: %s\n", #x, hipGetErrorString(e));         \
      exit(1);                                              \
    }                                                       \
  } while (0)

__global__ void k_read(const uint4* __restrict__ a, size_t n, unsigned* out) {
  unsigned s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

// the copy as a kernel: uint4 loads from device memory, uint4 stores into the mapped page-locked
// buffer (the CUs write across PCIe; no SDMA engine)
__global__ void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

int main(int argc, char** argv) {
  const int ns = argc > 1 ? atoi(argv[1]) : 12;
  const bool destroy = argc > 2 && argv[2][0] == 'd';
  const size_t cb = 64ull << 20, kb = 2ull << 30;
  void *d, *big, *h;
  unsigned* o;
  CK(hipMalloc(&d, cb));
  CK(hipMalloc(&big, kb));
  CK(hipMalloc(&o, 4));
  const char* where = argc > 3 ? argv[3] : "p";
  const int kgrid = argc > 4 ? atoi(argv[4]) : 0;  // > 0: copy by k_copy on that many workgroups
  unsigned flags = hipHostMallocPortable;
  const int node = gpu_node();
  if (strcmp(where, "p")) {
    bind_node(strcmp(where, "near") == 0 ? node : 1 - node);
    flags |= hipHostMallocNumaUser;
  }
  printf("gpu node %d, buffer: %s, copy: %s %d\n", node, where, kgrid ? "kernel" : "SDMA", kgrid);
  CK(hipHostMalloc(&h, cb, flags));
  CK(hipMemset(d, 0x5a, cb));
  CK(hipMemset(big, 1, kb));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, h));
  void* hd = at.devicePointer;
  for (int i = 0; i < ns; ++i) {
    hipStream_t s0, s1;
    CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    double ms[2];
    for (int busy = 0; busy < 2; ++busy) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      for (int r = 0; r < 10; ++r) {
        if (busy) hipLaunchKernelGGL(k_read, dim3(2048), dim3(256), 0, s0, (const uint4*)big, kb / 16, o);
        if (kgrid)
          hipLaunchKernelGGL(k_copy, dim3(kgrid), dim3(256), 0, s1, (const uint4*)d, (uint4*)hd, cb / 16);
        else
          CK(hipMemcpyAsync(hd, d, cb, hipMemcpyDeviceToDeviceNoCU, s1));
      }
      CK(hipStreamSynchronize(s1));
      ms[busy] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      CK(hipDeviceSynchronize());
    }
    printf("stream pair %2d: copies alone %6.1f GB/s, beside a kernel %6.1f GB/s\n", i, 10 * cb / ms[0] / 1e6,
           10 * cb / ms[1] / 1e6);
    fflush(stdout);
    if (destroy) {
      CK(hipStreamDestroy(s0));
      CK(hipStreamDestroy(s1));
    }
  }
  return 0;
}
