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

// ---- packed fact values (EL_STREAM_PACKED): code = the value's bit column when below CODE_ESC,
// else CODE_ESC with the value in the escape list (log order).  Passed to the fact log's run
// encoding, which then also counts the escapes per tile (cnt), writes codes[e] for e in [a, b)
// (below code_cap) and the escapes at esc[*base + off[t] + i] (below esc_cap), and advances
// *base / *total like the runs' own.
constexpr uint32_t CODE_ESC = 0xffffu;
struct Codes {
  const uint32_t* vals = nullptr;   // the log's values
  const uint32_t* cperm = nullptr;  // concept -> column (nullptr: the window in id order)
  uint32_t c_lo = 0, c_hi = 0;
  uint32_t* cnt = nullptr;          // escapes per tile (count) ...
  const uint32_t* off = nullptr;    // ... and their exclusive scan (emit)
  uint16_t* codes = nullptr;
  uint64_t code_cap = 0;
  uint32_t* esc = nullptr;
  uint64_t esc_cap = 0;
  unsigned long long* base = nullptr;
  unsigned long long* total = nullptr;
};

// cnt[t] = runs starting in tile t of keys[a, b)
void count(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, uint32_t* cnt, const Codes* pk = nullptr);
// the runs of keys[a, b) as (key, end) at out[*base + off[t] + i] (only those below cap; off =
// exclusive scan of cnt), then *base += Σ cnt and *total = *base (a one-thread launch behind the
// emit; total may be mapped host memory)
void emit(hipStream_t s, const uint32_t* keys, uint64_t a, uint64_t b, const uint32_t* off, const uint32_t* cnt,
          uint2* out, uint64_t cap, unsigned long long* base, unsigned long long* total, const Codes* pk = nullptr);

}  // namespace elst
