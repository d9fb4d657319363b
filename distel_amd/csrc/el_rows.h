// el_rows.h — row-sorted CSR of an append-only (row, value) log, built on the device.
//
// The result copy-back ("IR-in-HBM to fixpoint plus result copy-back")
// hands the caller the result node in its rearranged form X -> {B} (ResultRearranger DB1,
// ResultRearranger.java:57-105) and the role links X -> {(r, Y)}.  The engine keeps both as
// append-only logs in superstep order; this module turns a log into CSR rows, ascending within
// each row, without a host round trip:
//
//   k_rows_count    per-row counts + each entry's rank in its row (one atomic per run of equal
//                   rows in a wave: the log holds whole told closures back to back)
//   scan            uint64 row offsets (library scan)
//   k_rows_scatter  entry -> ptr[row] + rank (optionally through a value -> key map)
//   k_rows_small    rows of <= 64 entries: one register bitonic sort per row (a wave)
//   k_rows_lds      rows of <= 4096 entries: LDS bitonic sort, one workgroup per row
//   k_rows_bits     longer rows with a bit matrix: the row's set bits in order (no sort)
//   k_rows_global   longer rows without one: bitonic sort in global memory, one workgroup per row
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace elrows {

struct Scratch {
  uint32_t* rank = nullptr;  // per log entry
  uint64_t rank_cap = 0;
  uint32_t* cnt = nullptr;  // rows + 1
  uint64_t cnt_cap = 0;
  uint32_t* lists = nullptr;  // medium rows [0, rows), long rows [rows, 2 rows)
  uint64_t list_cap = 0;
  uint32_t* nlist = nullptr;  // two counters, 256 B apart
  void* cub = nullptr;
  size_t cub_bytes = 0;
  void release();
};

// Rows [row_lo, row_lo + R) of the log entries (rows[i], vals[i]), i < n (every rows[i] in
// range).  ptr: R + 1 offsets; out: n values, keymap ? keymap[v] : v, ascending in each row.
// bits (optional): virtual base of a bit matrix holding exactly the log's entries, row x at
// bits + x * W (values are column ids); long rows are then read from it instead of sorted.
// Everything is enqueued on `s`; nothing is read back.  Throws std::runtime_error on a HIP error.
void build(hipStream_t s, Scratch& sc, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t row_lo,
           uint32_t R, const uint32_t* keymap, uint64_t* ptr, uint32_t* out, const uint32_t* bits, uint64_t W);

}  // namespace elrows
