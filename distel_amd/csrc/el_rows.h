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
//   scan            uint64 row offsets (k_rows_tiles, k_rows_tile_scan, k_rows_offsets; the
//                   last also lists the rows longer than 64 entries)
//   k_rows_scatter  entry -> tmp[ptr[row] + rank] (optionally through a value -> key map)
//   k_rows_small    rows of <= 64 entries: register bitonic sort per row (a wave) -> dst
//   k_rows_lds      rows of <= 4096 entries: LDS bitonic sort, one workgroup per row -> dst
//   k_rows_bits     longer rows with a bit matrix: the row's set bits in order (no sort) -> dst
//   k_rows_global   longer rows without one: bitonic sort in place in tmp, then -> dst
//   k_rows_readout  every row of a bit matrix, read off in column order (the S rows of a
//                   large copy-back: build_counts + readout, chunked behind DMAs)
//
// dst may be device memory or page-locked host memory mapped for the device: the sort
// kernels then write the sorted rows straight over PCIe (the copy-back is fused with the sort,
// no device staging copy and no separate DMA).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

// Block summary granularity: one summary byte per 2^EL_SUMM_SHIFT bits of a matrix row (12: a
// 512-B block, 9: a 64-B line).  The read-out works in 512-B blocks (the OR of SUMM_SUB bytes).
#ifndef EL_SUMM_SHIFT
#define EL_SUMM_SHIFT 9
#endif
static_assert(EL_SUMM_SHIFT >= 9 && EL_SUMM_SHIFT <= 12, "summary block: 64 B .. 512 B");

namespace elrows {

constexpr uint32_t SUMM_SHIFT = EL_SUMM_SHIFT;
constexpr uint32_t SUMM_WORDS = 1u << (SUMM_SHIFT - 5);   // matrix words per summary byte
constexpr uint32_t SUMM_SUB = 1u << (12 - SUMM_SHIFT);     // summary bytes per 512-B block

// The S bit matrix: row x at bits + x·W, rows r of the build at x = r + lo; columns ⊥, ⊤,
// then the concepts [c_lo, c_hi) (column c >= 2 is concept c + c_lo - 2).  Read by the
// long-row read-out; cleared as the rows are written when the caller releases its state.
// bits = nullptr: no matrix.
struct Clear {
  uint32_t* bits = nullptr;
  uint64_t W = 0;
  uint32_t lo = 0;
  uint32_t c_lo = 2, c_hi = 0xffffffffu;
  // optional block summary: byte x·SB + k is non-zero if row x may hold a set bit in its block k
  // (words [SUMM_WORDS k, SUMM_WORDS (k + 1))); the read-out then reads only the 512-B blocks
  // whose SUMM_SUB bytes are not all zero
  uint8_t* summ = nullptr;  // (the read-out zeroes a row's bytes with its words when clearing)
  uint32_t SB = 0;
  __device__ void bit(uint32_t r, uint32_t v) const;
};

struct Scratch {
  uint32_t* rank = nullptr;  // per log entry
  uint64_t rank_cap = 0;
  uint32_t* tmp = nullptr;  // scattered (unsorted) rows, per log entry
  uint64_t tmp_cap = 0;
  uint32_t* cnt = nullptr;  // rows + 1
  uint64_t cnt_cap = 0;
  uint32_t* lists = nullptr;  // medium rows [0, rows), long rows [rows, 2 rows)
  uint64_t list_cap = 0;
  uint32_t* nlist = nullptr;  // two counters, 256 B apart
  uint64_t* tile = nullptr;  // scan tile sums
  uint64_t tile_cap = 0;
  uint64_t n = 0;      // the prepared build (build_prep -> build_sort)
  uint32_t R = 0;
  bool bits = false;
  void release();
};

// Rows [row_lo, row_lo + R) of the log entries (rows[i], vals[i]), i < n (entries of other
// rows are left out).  ptr (device): R + 1 offsets; dst: n values, keymap ? keymap[v] : v, ascending in
// each row (device memory, or host memory the device can write).  vals = nullptr: the value
// of entry i is i (rows of log indices).
// matrix (optional): a bit matrix holding exactly the log's entries (values are concept ids);
// long rows are then read from it instead of sorted.
// Everything is enqueued on `s`; nothing is read back.  Throws std::runtime_error on a HIP error.
void build(hipStream_t s, Scratch& sc, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t row_lo,
           uint32_t R, const uint32_t* keymap, uint64_t* ptr, uint32_t* dst, Clear matrix);

// build() in two halves: build_prep reads the log (and the bit matrix for the long rows);
// build_sort reads only the scratch, so the log's owner may reuse its state once the prep's
// work has completed on s.  clear (prep) / cl (sort): zero the matrix bits of the written
// entries as they go, leaving the matrix empty (the caller is done with it).
void build_prep(hipStream_t s, Scratch& sc, const uint32_t* rows, const uint32_t* vals, uint64_t n, uint32_t row_lo,
                uint32_t R, const uint32_t* keymap, uint64_t* ptr, uint32_t* dst, Clear matrix, bool clear);
void build_sort(hipStream_t s, Scratch& sc, const uint64_t* ptr, uint32_t* dst, Clear cl);

// Row offsets only (counts of the log's rows, scanned): ptr (device), R + 1 entries.
void build_counts(hipStream_t s, Scratch& sc, const uint32_t* rows, uint64_t n, uint32_t row_lo, uint32_t R,
                  uint64_t* ptr);
// Rows [r0, r1) of a bit matrix whose rows hold exactly the counted entries (ptr from
// build_counts over the same log), read off the matrix in column order — sorted without a
// sort — into dst[ptr[r] - out0 ...] (device memory); clear zeroes the words read.  W must be a
// multiple of 4 (rows 16-B aligned).
void readout(hipStream_t s, const uint64_t* ptr, uint32_t r0, uint32_t r1, uint64_t out0, uint32_t* dst, Clear m,
             bool clear);

}  // namespace elrows
