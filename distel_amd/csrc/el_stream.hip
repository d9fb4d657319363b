// el_stream.hip — run encoding of the streamed result's log segments (el_stream.h).
#include "el_stream.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace elst {
namespace {

#define SCHK(expr)                                                                        \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr uint32_t WAVES = BLOCK / 64;

uint32_t grid(uint64_t nt) { return (uint32_t)(nt < 1024 ? (nt ? nt : 1) : 1024); }

// A run starts at e when e opens its tile or its key differs from the one before.
__device__ __forceinline__ bool run_head(const uint32_t* __restrict__ keys, uint64_t e, uint64_t t0, uint32_t key) {
  return e == t0 || keys[e - 1] != key;
}

__global__ void __launch_bounds__(BLOCK) k_run_count(const uint32_t* __restrict__ keys, uint64_t a, uint64_t b,
                                                     uint32_t* __restrict__ cnt) {
  __shared__ uint32_t wsum[WAVES];
  const uint64_t nt = tiles(b - a);
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {  // (block-uniform trip count)
    const uint64_t t0 = a + t * TILE, t1 = min(b, t0 + TILE);
    uint32_t c = 0;
    for (uint32_t k = 0; k < ITEMS; ++k) {
      const uint64_t e = t0 + (uint64_t)k * BLOCK + threadIdx.x;
      if (e < t1) c += run_head(keys, e, t0, keys[e]) ? 1u : 0u;
    }
    for (uint32_t o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if (lane == 0) wsum[w] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t s = 0;
      for (uint32_t i = 0; i < WAVES; ++i) s += wsum[i];
      cnt[t] = s;
    }
    __syncthreads();
  }
}

// Tile t's runs are numbered from base + off[t] in log order: the run of a tail element e (the
// last of its run in the tile) is the number of heads up to e, minus one.  Coalesced loads
// (element k·BLOCK + thread of the tile), one ballot per round for the heads.
__global__ void __launch_bounds__(BLOCK) k_run_emit(const uint32_t* __restrict__ keys, uint64_t a, uint64_t b,
                                                    const uint32_t* __restrict__ off, uint2* out, uint64_t cap,
                                                    const unsigned long long* base) {
  __shared__ uint32_t wtot[WAVES];
  const uint64_t nt = tiles(b - a), b0 = *base;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (uint64_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const uint64_t t0 = a + t * TILE, t1 = min(b, t0 + TILE);
    const uint64_t run0 = b0 + off[t];
    uint32_t running = 0;  // heads of the tile before this round
    for (uint32_t k = 0; k < ITEMS; ++k) {
      const uint64_t e = t0 + (uint64_t)k * BLOCK + threadIdx.x;
      const bool valid = e < t1;
      const uint32_t key = valid ? keys[e] : 0u;
      const bool head = valid && run_head(keys, e, t0, key);
      const bool tail = valid && (e + 1 == t1 || keys[e + 1] != key);
      const unsigned long long m = __ballot(head);
      if (lane == 0) wtot[w] = (uint32_t)__popcll(m);
      __syncthreads();
      uint32_t before = 0, all = 0;
      for (uint32_t i = 0; i < WAVES; ++i) {
        const uint32_t v = wtot[i];
        before += i < w ? v : 0u;
        all += v;
      }
      __syncthreads();  // (wtot is rewritten next round)
      if (tail) {
        const uint64_t r = run0 + running + before + (uint32_t)__popcll(m & below) + (head ? 1u : 0u) - 1u;
        if (r < cap) out[r] = make_uint2(key, (uint32_t)(e + 1));
      }
      running += all;
    }
  }
}

__global__ void k_run_advance(unsigned long long* base, const uint32_t* off, const uint32_t* cnt, uint64_t last,
                              unsigned long long* total) {
  const unsigned long long v = *base + off[last] + cnt[last];
  *base = v;
  *total = v;
}

}  // namespace

void count(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, uint32_t* cnt) {
  if (b <= a) return;
  hipLaunchKernelGGL(k_run_count, dim3(grid(tiles(b - a))), dim3(BLOCK), 0, s, keys, a, b, cnt);
  SCHK(hipGetLastError());
}

void emit(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, const uint32_t* off, const uint32_t* cnt,
          uint2* out, uint64_t cap, unsigned long long* base, unsigned long long* total) {
  if (b <= a) return;
  const uint64_t nt = tiles(b - a);
  hipLaunchKernelGGL(k_run_emit, dim3(grid(nt)), dim3(BLOCK), 0, s, keys, a, b, off, out, cap, base);
  SCHK(hipGetLastError());
  hipLaunchKernelGGL(k_run_advance, dim3(1), dim3(1), 0, s, base, off, cnt, nt - 1, total);
  SCHK(hipGetLastError());
}

// ---- SDMA copies through HSA

struct Sdma::Impl {
  hsa_agent_t gpu{}, cpu{};
  uint32_t engine = 0;  // an HSA_AMD_SDMA_ENGINE_* bit
  std::vector<hsa_signal_t> pool, pending;
  bool hsa_up = false;
};

namespace {
struct Found {
  uint32_t domain = 0, bdf = 0;
  bool have_gpu = false, have_cpu = false;
  hsa_agent_t gpu{}, cpu{};
};
hsa_status_t find_agents(hsa_agent_t a, void* data) {
  Found* f = static_cast<Found*>(data);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
    f->cpu = a;
    f->have_cpu = true;
  } else if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) {
    uint32_t bdf = 0, dom = 0;
    if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
        bdf == f->bdf && dom == f->domain) {
      f->gpu = a;
      f->have_gpu = true;
    }
  }
  return HSA_STATUS_SUCCESS;
}
}  // namespace

Sdma::Sdma(int hip_device) : impl_(new Impl) {
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, hip_device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, hip_device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, hip_device) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if (hsa_init() != HSA_STATUS_SUCCESS) return;  // (reference-counted: HIP initialised it already)
  impl_->hsa_up = true;
  Found f;
  f.domain = (uint32_t)dom;
  f.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);  // function 0
  if (hsa_iterate_agents(find_agents, &f) != HSA_STATUS_SUCCESS || !f.have_gpu || !f.have_cpu) return;
  impl_->gpu = f.gpu;
  impl_->cpu = f.cpu;
  uint32_t mask = 0;
  if (hsa_amd_memory_get_preferred_copy_engine(f.cpu, f.gpu, &mask) != HSA_STATUS_SUCCESS || mask == 0)
    if (hsa_amd_memory_copy_engine_status(f.cpu, f.gpu, &mask) != HSA_STATUS_SUCCESS) mask = 0;
  if (mask == 0) return;
  impl_->engine = mask & (~mask + 1u);  // the lowest engine offered
  ok_ = true;
}

Sdma::~Sdma() {
  if (!impl_) return;
  try {
    wait();
  } catch (...) {
  }
  for (hsa_signal_t s : impl_->pool) (void)hsa_signal_destroy(s);
  if (impl_->hsa_up) (void)hsa_shut_down();
  delete impl_;
}

void Sdma::copy(void* dst_host, const void* src_dev, size_t bytes) {
  if (!bytes) return;
  hsa_signal_t sig;
  if (!impl_->pool.empty()) {
    sig = impl_->pool.back();
    impl_->pool.pop_back();
    hsa_signal_store_screlease(sig, 1);
  } else if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) {
    throw std::runtime_error("hsa_signal_create failed");
  }
  const hsa_status_t st = hsa_amd_memory_async_copy_on_engine(
      dst_host, impl_->cpu, src_dev, impl_->gpu, bytes, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)impl_->engine, true);
  if (st != HSA_STATUS_SUCCESS) {
    impl_->pool.push_back(sig);
    throw std::runtime_error("hsa_amd_memory_async_copy_on_engine failed (" + std::to_string((int)st) + ")");
  }
  impl_->pending.push_back(sig);
  pending_n_ = impl_->pending.size();
}

void Sdma::wait() {
  for (hsa_signal_t s : impl_->pending) {
    while (hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
    }
    impl_->pool.push_back(s);
  }
  impl_->pending.clear();
  pending_n_ = 0;
}

}  // namespace elst
