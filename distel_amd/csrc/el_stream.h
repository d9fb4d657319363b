// el_stream.h — run encoding of the streamed result (el_stream_result).
//
// The fact log holds (x, b) in commit order and the link log (x, pid); the commit stages new
// entries per block and wave, and the init facts / base links are written in x order, so x
// comes in long runs.  Each committed segment of a log crosses PCIe as its values (b, or pid:
// one DMA) plus its runs (x, end): entries [end of the previous run, end) belong to row x.  The
// runs are found on the device (a tile count, a scan of the counts, an emit) and written in
// log order into a device run buffer that follows the values by DMA, so the host receives 4 B
// per entry plus 8 B per run instead of 8 B per entry.  A tile start always starts a run,
// so both passes see the same runs without looking across tiles.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace elst {

constexpr uint32_t BLOCK = 256;
constexpr uint32_t ITEMS = 8;
constexpr uint32_t TILE = BLOCK * ITEMS;

__host__ __device__ inline uint64_t tiles(uint64_t n) { return (n + TILE - 1) / TILE; }

// cnt[t] = runs starting in tile t of keys[a, b)
void count(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, uint32_t* cnt);
// the runs of keys[a, b) as (key, end) at out[*base + off[t] + i] (only those below cap; off =
// exclusive scan of cnt), then *base += Σ cnt and *total = *base (a one-thread launch behind the
// emit; total may be mapped host memory)
void emit(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, const uint32_t* off, const uint32_t* cnt,
          uint2* out, uint64_t cap, unsigned long long* base, unsigned long long* total);

}  // namespace elst
