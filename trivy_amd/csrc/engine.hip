// MI355X (gfx950) secret-scanning engine: two HIP kernels + host driver.
//
// K1  tsg_k1_scan    one streaming pass over the packed batch in HBM.  Each
//                    thread owns a CHUNK of bytes (16-byte vector loads),
//                    warms its DFA state up over the preceding
//                    (max_pattern_bytes-1) bytes of the same file, then steps
//                    the LDS-resident scan DFA (keyword + anchor literals,
//                    uint16 transitions over byte classes) byte by byte.
//                    Keyword outputs set per-(file, keyword) bits (exact
//                    bytes.ToLower gate, scanner.go:174-186); anchor outputs
//                    append a 64-bit hit (end offset << 24 | anchor id).  It
//                    also counts '\n' per chunk (newline prefix for line
//                    numbers).  Memory-bound target: HBM, 1 byte read per
//                    content byte.
// K2  tsg_k2_verify  one thread per anchor hit: keyword gate of the hit's
//                    rule, then the rule's anchored relaxed verify DFA (L2
//                    resident) from every possible match start in the
//                    anchor's offset window.  Accepting starts become
//                    (file, rule, start) candidates for the host confirmer.
// No MFMA anywhere: this path is byte/integer automaton work.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <thread>

#include "crstrip.h"
#include "engine.h"
#include "pipeline.h"
#include "threadpool.h"

namespace tsg {

namespace {

constexpr uint32_t kLdsBytes = 160 * 1024;     // LDS per CU

struct CandDev { uint32_t file, rule; unsigned long long start; };

// Readback of a segment's results into host-mapped, fine-grained pinned
// memory with plain vector stores over PCIe: no copy engine, so a readback
// never queues behind an upload, and no DMA setup latency per small copy.
// One launch moves up to kRbMax regions (blockIdx.y selects one): region k
// copies nwords dwords, or min(*count * per_count, nwords) with a count
// (16-byte granules: both buffers carry slack past the end).  (A launch per
// region cost ~4 us of dispatch each on small segments: per-file batches.)
constexpr int kRbMax = 5;
struct RbRegion { const uint4* src; uint4* dst; const uint32_t* count; uint32_t nwords, per_count; };
struct RbList { RbRegion r[kRbMax]; };
__global__ __launch_bounds__(256) void tsg_readback(RbList L) {
  const RbRegion& g = L.r[blockIdx.y];
  uint32_t n = g.nwords;
  if (g.count) n = static_cast<uint32_t>(min(static_cast<unsigned long long>(n),
                                             static_cast<unsigned long long>(*g.count) * g.per_count));
  const uint32_t n4 = (n + 3) / 4;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += gridDim.x * 256) g.dst[i] = g.src[i];
}

// A segment's prologue in one launch: zeroes up to four dword ranges (K1's
// per-segment scratch: keyword bits, file flags, counters, per-region hit
// counts; four memsets were four dispatches) and, for a small batch in
// pinned host memory, copies its bytes and offsets into the lane's buffers
// over PCIe itself (blockIdx.y 4 and 5) -- no copy-engine upload and no
// cross-stream wait in front of K1 (~25 us of a one-file batch), with the
// 64 bytes past the data zeroed (K1 reads 16-byte words past the end).
struct Prologue {
  uint32_t* p[4];
  uint32_t n[4];
  const uint8_t* src[2];       // device view of pinned host memory
  uint8_t* dst[2];
  uint32_t bytes[2];
  uint32_t zpad[2];            // bytes to zero after the copy
};
__global__ __launch_bounds__(256) void tsg_prologue(Prologue L) {
  const uint32_t y = blockIdx.y;
  const uint32_t tid = blockIdx.x * 256 + threadIdx.x, step = gridDim.x * 256;
  if (y < 4) {
    uint32_t* p = L.p[y];
    for (uint32_t i = tid; i < L.n[y]; i += step) p[i] = 0;
    return;
  }
  const uint8_t* src = L.src[y - 4];
  uint8_t* dst = L.dst[y - 4];
  const uint32_t n = L.bytes[y - 4];
  uint32_t done = 0;
  if ((reinterpret_cast<uintptr_t>(src) & 15u) == 0) {
    const uint32_t n16 = n / 16;
    for (uint32_t i = tid; i < n16; i += step)
      reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    done = n16 * 16;
  }
  for (uint32_t i = done + tid; i < n; i += step) dst[i] = src[i];
  for (uint32_t i = tid; i < L.zpad[y - 4]; i += step) dst[n + i] = 0;
}

#define HIP_OK(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      if (err) *err = std::string(#expr) + ": " + hipGetErrorString(e_);          \
      return false;                                                               \
    }                                                                             \
  } while (0)

__device__ __forceinline__ uint32_t file_of(const uint64_t* __restrict__ off, uint32_t nfiles, uint64_t pos) {
  // largest f with off[f] <= pos, then skip empty files (off[f+1] == off[f])
  uint32_t lo = 0, hi = nfiles;   // search in off[0..nfiles]
  while (lo < hi) {
    uint32_t m = (lo + hi + 1) >> 1;
    if (off[m] <= pos) lo = m; else hi = m - 1;
  }
  uint32_t f = lo;
  while (f < nfiles && off[f + 1] <= pos) ++f;
  return f;
}

// K1's file index (round 6): fidx[b] = file_of(b << kFidxShift) for every
// 64 KiB block of the launch, built by tsg_file_index before K1, so a range
// start's file is a binary search between two neighbouring entries (0-3
// dependent loads for large files) instead of over every file (11-19): the
// items after a wave's first took ~9 us to set up under K1's memory load
// against ~3 us for the first (profiles/r7z_k1_trace_c2_step.txt).
constexpr uint32_t kFidxShift = 16;
__global__ __launch_bounds__(256) void tsg_file_index(const uint64_t* __restrict__ off, uint32_t nfiles,
                                                      uint32_t* __restrict__ fidx, uint32_t nblk) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b < nblk) fidx[b] = file_of(off, nfiles, static_cast<uint64_t>(b) << kFidxShift);
}
// file_of(off, nfiles, pos) for pos < off[nfiles], searched between the index
// entries of pos's block and the next one (file_of is monotonic in pos)
__device__ __forceinline__ uint32_t file_of_idx(const uint64_t* __restrict__ off, uint32_t nfiles,
                                                const uint32_t* __restrict__ fidx, uint64_t pos) {
  const uint64_t b = pos >> kFidxShift;
  uint32_t lo = fidx[b], hi = min(fidx[b + 1], nfiles);
  while (lo < hi) {
    const uint32_t m = (lo + hi + 1) >> 1;
    if (off[m] <= pos) lo = m; else hi = m - 1;
  }
  uint32_t f = lo;
  while (f < nfiles && off[f + 1] <= pos) ++f;
  return f;
}

constexpr uint32_t kWaveHits = kK1WaveHits;   // largest per-wave LDS hit buffer (entries of 4 bytes: offset in item << 11 | anchor)
constexpr uint32_t kAnchorBits = 11;   // anchors per ruleset < 2048 (checked on the host)
constexpr uint32_t kMaxWaves = 16;     // K1 workgroups are at most 1024 threads
constexpr double kDenseFilesPerGB = 8000.0;   // upload segmentation: "many small files" (image layers: ~48k/GB)
// per-lane device counters: [0] cands, [1] K2 count, [2] overflow, [3] LDS-base
// error, [4 + g] K1 items of group g
constexpr size_t kCntBytes = 8192;
// K1's work-item counters: group g's at dword kItemCtrBase + g * 256, eight
// of them 32 dwords (one 128-byte line) apart, one per XCD
constexpr uint32_t kItemCtrBase = 256, kMaxK1Groups = 7;
constexpr size_t kInlineConfirmFiles = 4;          // confirmations this small run on the calling thread
constexpr uint64_t kInlineConfirmBytes = 512 << 10;
constexpr int kItemChunks = 4;         // a K1 wave item: 64 lanes x (up to) 4 chunks

// Largest K1 chunk whose wave item (64 lanes x kS chunks) fits the LDS hit
// record's 32 - kAnchorBits offset bits.
constexpr uint32_t k1_max_chunk(int ks) {
  return ((1u << (32 - kAnchorBits)) / (64u * static_cast<uint32_t>(ks))) & ~127u;
}
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// Keyword ids < 128 accumulate in two per-stream 64-bit masks, flushed with
// atomicOr at file changes and at the end of the stream's chunk.
// Most chunks of a file repeat keywords an earlier chunk already set, and many
// lanes OR into the same words of a large file: read first, and only issue
// the (memory-side, serialising) atomic for bits not yet visible.  A stale
// read only costs a redundant atomic.
__device__ __forceinline__ void or_bits(uint32_t* w, uint32_t bits) {
  if (bits && (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & bits) != bits) atomicOr(w, bits);
}

// At a file boundary inside a lane's range: no-return atomics only (the
// lane's next file starts at once; a read-first or_bits would stall the whole
// wave on an L2 round trip per word at every boundary)
__device__ __forceinline__ void flush_kw_blind(uint32_t* __restrict__ kwbits, uint32_t kw_words, uint32_t f,
                                               unsigned long long& kw0, unsigned long long& kw1) {
  uint32_t* w = kwbits + static_cast<size_t>(f) * kw_words;
  if (static_cast<uint32_t>(kw0)) atomicOr(w + 0, static_cast<uint32_t>(kw0));
  if (static_cast<uint32_t>(kw0 >> 32)) atomicOr(w + 1, static_cast<uint32_t>(kw0 >> 32));
  if (static_cast<uint32_t>(kw1)) atomicOr(w + 2, static_cast<uint32_t>(kw1));
  if (static_cast<uint32_t>(kw1 >> 32)) atomicOr(w + 3, static_cast<uint32_t>(kw1 >> 32));
  kw0 = kw1 = 0;
}

__device__ __forceinline__ void flush_kw(uint32_t* __restrict__ kwbits, uint32_t kw_words, uint32_t f,
                                         unsigned long long& kw0, unsigned long long& kw1) {
  uint32_t* w = kwbits + static_cast<size_t>(f) * kw_words;
  if (kw0) {
    or_bits(w + 0, static_cast<uint32_t>(kw0));
    or_bits(w + 1, static_cast<uint32_t>(kw0 >> 32));
  }
  if (kw1) {
    or_bits(w + 2, static_cast<uint32_t>(kw1));
    or_bits(w + 3, static_cast<uint32_t>(kw1 >> 32));
  }
  kw0 = kw1 = 0;
}

// exact count of 0x0a bytes in a 32-bit word
__device__ __forceinline__ uint32_t nl_in_word(uint32_t w) {
  const uint32_t x = w ^ 0x0a0a0a0au;
  const uint32_t y = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
  return __popc(y);
}

// Per-stream state of K1.  A lane walks kS independent byte ranges (streams)
// with their transition chains interleaved, so the LDS latency of one
// dependent chain hides behind the others.  A stream starts on the 128-byte
// line at or before (chunk start - warm-up): the bytes before the chunk only
// warm the DFA up (no outputs, no newline counts); the chunk's own bytes
// start at `emit`.  Starting earlier than needed is harmless: the scan DFA's
// state depends only on the last max_pattern_bytes - 1 bytes of the file.
struct K1Stream {
  unsigned long long p, lim, emit;   // next byte; min(stream end, file end); first byte with outputs
  unsigned long long end;            // stream end: the lane's range of chunks
  unsigned long long cend;           // v3: end of the current chunk (its '\n' count is stored there)
  unsigned long long ci;             // v3: index of the current chunk
  uint32_t f, s, p12, nl;            // file; DFA row offset; previous two bytes (p1 | p2 << 8); newlines
  unsigned long long kw0, kw1;
};

// Output metadata of a state with outputs, in LDS: its keyword ids < 128 as
// two masks, and a list of the other output ids (anchors, keywords >= 128).
struct OutMeta { unsigned long long kw0, kw1; uint32_t list_begin, list_count; };

struct K1Ctx {
  const uint8_t* __restrict__ data;
  unsigned long long total;
  uint32_t chunk;
  const uint64_t* __restrict__ offsets;
  uint32_t nfiles;
  const uint32_t* __restrict__ fidx;   // the launch's file index (tsg_file_index), or nullptr
  const uint16_t* next;   // pre-multiplied: next[s + c] is the next state's row offset
  const uint8_t* cls;     // byte -> class * 2
  uint32_t first_out;     // row offset (dwords) of the first state with outputs
  uint32_t wave_hits;     // per-wave LDS hit buffer entries of this launch
  uint32_t nclasses;      // row slot `nclasses` holds the output-state index
  const OutMeta* meta;
  const uint32_t* list;
  uint32_t nkw;
  uint32_t* __restrict__ kwbits;
  uint32_t* __restrict__ kwmask;  // kwbits + kw_base / 32: the register masks' first word
  uint32_t kw_words;
  bool primary;                   // first scan group: also counts newlines and flags fold-special files
  unsigned long long* __restrict__ hits;   // this workgroup's region of the hit list
  uint32_t region_cap;
  unsigned long long* __restrict__ over;   // shared overflow pool for hits past a full region
  uint32_t* over_cnt;
  uint32_t over_cap;
  uint32_t* b_hitcnt;           // LDS: fill count of the workgroup's region
  uint32_t* w_hits;             // this wave's LDS hit buffer
  unsigned long long item_base; // first byte of the wave's current item
  uint32_t* w_hitcnt;           // and its fill count
  uint32_t* __restrict__ fflags;
  uint32_t s0;                  // the start state's value: 0 (K1), the start's packed value (K1c)
};

// One transition: `s` is the current state's row offset (state * stride, in
// uint16 elements) and `c2` the byte's class times 2 (the class map is stored
// pre-doubled) and rows start on dwords, so the LDS byte address is
// (s << 2) + c2 with `s` the row offset in dwords (tables up to 256 KiB).
__device__ __forceinline__ uint32_t k1_step(const uint16_t* next, uint32_t s, uint32_t c2) {
  return *reinterpret_cast<const uint16_t*>(reinterpret_cast<const uint8_t*>(next) + ((s << 2) + c2));
}

// LDS reads by integer LDS address: the kernel's dynamic LDS starts
// at offset 0 (no static LDS; checked at run time by k1_lds_base_ok), so a
// transition address is one v_lshl_add_u32 feeding a ds_read_u16 whose
// immediate offset is the table's position.
typedef __attribute__((address_space(3))) const uint16_t k1_lds16_t;
typedef __attribute__((address_space(3))) const uint8_t k1_lds8_t;
__device__ __forceinline__ uint32_t k1_lds16(uint32_t a) { return *reinterpret_cast<k1_lds16_t*>(a); }
__device__ __forceinline__ uint32_t k1_lds8(uint32_t a) { return *reinterpret_cast<k1_lds8_t*>(a); }
typedef __attribute__((address_space(3))) const uint32_t k1_lds32_t;
typedef __attribute__((address_space(3))) const v4u k1_lds128_t;
__device__ __forceinline__ uint32_t k1_lds32(uint32_t a) { return *reinterpret_cast<k1_lds32_t*>(a); }
__device__ __forceinline__ v4u k1_lds128(uint32_t a) { return *reinterpret_cast<k1_lds128_t*>(a); }

// K1c step (prefilter.h CompressedScan): the row entry and the DESC record are
// both addressed from the packed state, so the two LDS reads issue together;
// the record's four class slots (class * 4, 0xff = none) pick target A (slots
// 0-1), target B (slots 2-3) or the row entry.  rep = c4 * 0x01010101.
__device__ __forceinline__ uint32_t k1c_next(uint32_t s, uint32_t c4, uint32_t rep) {
  const uint32_t f = k1_lds32(((s >> 16) << 2) + c4);
  const v4u d = k1_lds128(s & 0xfff0u);
  const uint32_t x = d.x ^ rep;
  const uint32_t z = (x - 0x01010101u) & ~x & 0x80808080u;
  return (z & 0x8080u) ? d.y : ((z & 0x80800000u) ? d.z : f);
}
__device__ __forceinline__ bool k1_lds_base_ok(const uint8_t* smem) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((k1_lds8_t*)(smem))) == 0;
}

__device__ __forceinline__ unsigned long long k1_end(const K1Ctx& x, const K1Stream& t) { return t.end; }

// U+0130 / U+017F / U+212A fold onto ASCII letters: flag every file that
// overlaps a 16-byte word ending such a sequence (host re-scans it exactly).
// A superset is safe (a flagged file is only scanned more carefully).
__device__ __forceinline__ void k1_special(const K1Ctx& x, const K1Stream& t, const v4u w,
                                           unsigned long long fend, unsigned long long end) {
  uint32_t a = t.p12 & 0xffu, bb = t.p12 >> 8;
  bool hit = false;
  for (int k = 0; k < 16 && t.p + k < end; ++k) {
    const uint32_t wk = (k & 8) ? ((k & 4) ? w.w : w.z) : ((k & 4) ? w.y : w.x);   // (no indexed array: scratch)
    const uint32_t b = (wk >> ((k & 3) * 8)) & 0xffu;
    if (t.p + k == fend) { a = bb = 0; }
    if ((b == 0xB0u && a == 0xC4u) || (b == 0xBFu && a == 0xC5u) || (b == 0xAAu && a == 0x84u && bb == 0xE2u)) hit = true;
    bb = a;
    a = b;
  }
  if (hit) {
    for (unsigned long long q = t.p; q < min(t.p + 16, end); ++q) atomicOr(&x.fflags[file_of(x.offsets, x.nfiles, q)], 1u);
  }
}

// The outputs of output state `st` (row offset): its row carries the keyword
// masks and the list position inline after the spare slot (S = silent-row
// stride), so one LDS round trip fetches them.
__device__ __forceinline__ void k1_out_v3(const K1Ctx& x, K1Stream& t, uint32_t st, unsigned long long q, uint32_t S) {
  const uint32_t* m = reinterpret_cast<const uint32_t*>(x.next + S) + st;   // st in dwords; 4-byte aligned: S is even
  const uint32_t a0 = m[0], a1 = m[1], a2 = m[2], a3 = m[3], li = m[4];
  t.kw0 |= (static_cast<unsigned long long>(a1) << 32) | a0;
  t.kw1 |= (static_cast<unsigned long long>(a3) << 32) | a2;
  const uint32_t begin = li & 0xffffu, count = li >> 16;
  for (uint32_t j = 0; j < count; ++j) {
    const uint32_t id = x.list[begin + j];
    if (id < x.nkw) {
      atomicOr(x.kwbits + static_cast<size_t>(t.f) * x.kw_words + (id >> 5), 1u << (id & 31));
    } else {
      const uint32_t li2 = atomicAdd(x.w_hitcnt, 1u);
      if (li2 < x.wave_hits) {
        x.w_hits[li2] = (static_cast<uint32_t>(q - x.item_base) << kAnchorBits) | (id - x.nkw);
      } else {                                           // buffer full: straight to the region
        const uint32_t gi = atomicAdd(x.b_hitcnt, 1u);
        if (gi < x.region_cap) {
          x.hits[gi] = (q << 24) | (id - x.nkw);
        } else {                                         // region full: the shared overflow pool
          const uint32_t oi = atomicAdd(x.over_cnt, 1u);
          if (oi < x.over_cap) x.over[oi] = (q << 24) | (id - x.nkw);
        }
      }
    }
  }
}

// K1c outputs of output state `st` (packed value; only its DESC address is
// used): the record's output index selects an OutMeta in global memory
// (L2-resident; K1c keeps every LDS byte for the table).
__device__ __forceinline__ void k1_out_c(const K1Ctx& x, K1Stream& t, uint32_t st, unsigned long long q) {
  const uint32_t oi = k1_lds32((st & 0xfff0u) + 12u);
  const OutMeta m = x.meta[oi];
  t.kw0 |= m.kw0;
  t.kw1 |= m.kw1;
  for (uint32_t j = 0; j < m.list_count; ++j) {
    const uint32_t id = x.list[m.list_begin + j];
    if (id < x.nkw) {
      or_bits(x.kwbits + static_cast<size_t>(t.f) * x.kw_words + (id >> 5), 1u << (id & 31));
    } else {
      const uint32_t li2 = atomicAdd(x.w_hitcnt, 1u);
      if (li2 < x.wave_hits) {
        x.w_hits[li2] = (static_cast<uint32_t>(q - x.item_base) << kAnchorBits) | (id - x.nkw);
      } else {
        const uint32_t gi = atomicAdd(x.b_hitcnt, 1u);
        if (gi < x.region_cap) {
          x.hits[gi] = (q << 24) | (id - x.nkw);
        } else {
          const uint32_t oi2 = atomicAdd(x.over_cnt, 1u);
          if (oi2 < x.over_cap) x.over[oi2] = (q << 24) | (id - x.nkw);
        }
      }
    }
  }
}

// measurement / layout bits for file boundaries inside a lane's range:
// kAblBndRead keeps the read-first keyword flush (rounds 1-4; valid results);
// kAblBndNoFlush drops the flush (invalid results: prices it)
constexpr int kAblBndRead = 65536, kAblBndNoFlush = 131072;
// measurement (results valid): per-workgroup and per-item wall-clock stamps
// (s_memrealtime, 100 MHz) in the slack half of the deferred-output buffer,
// copied to $TSG_K1_TRACE_FILE by the probe library (tools/k1_trace.py)
constexpr int kAblTrace = 262144;
// measurement (results valid): every item, the first of each wave included,
// from the global counter (rounds 1-5).  Default since round 6: a wave's
// first item is its own index in the grid, so the launch does not start with
// every wave's atomic on one address (the traces put ~37 us of each
// first-round item there: 4096 same-address atomics serialised in L2)
constexpr int kAblAtomicFirst = 524288;
// measurement (results valid): the items after the first round from one
// counter (until round 6).  Default: eight counters, one per XCD (workgroup
// index mod 8) on lines of their own, each handing out every eighth item, so
// the burst of waves finishing their first items together spreads over eight
// L2 lines instead of queueing on one (250 MB launch 0.1695 -> 0.160 ms,
// 1 GB 0.440 -> 0.433, 4 GB unchanged; profiles/r7n_*)
constexpr int kAblOneCounter = 1048576;
// layout bit (results valid; VERDICT r5 item 1a, root bypass): bit 0 of the
// LDS class map (classes are stored doubled, so it is free) flags the classes
// that keep the start state at the start state; a lane at the start state on
// such a byte skips its transition read (it drops out of that ds_read under
// EXEC, so fewer lanes contend for the banks).  The class map stays one byte
// per entry: tools/lds_bank_sim.py prices the transition read 5.50 -> 4.61
// LDS cycles per byte with no change to the class read.
constexpr int kAblRootSkip = 2097152;
// measurement (results valid): fast lines with a C4 / C5 / E2 lead byte are
// checked for the fold-special sequences by re-reading the line from memory
// byte by byte (rounds 4-5) instead of word by word (k1_line_special_words)
constexpr int kAblSpecialMem = 4194304;
constexpr uint32_t kTraceItemCap = 1u << 17;
constexpr uint32_t kTraceItemWords = 8;   // [start, end, kU << 24 | wg << 8 | wave, setup done, loop done, flushed, 0, 0]

// One 16-byte word of one stream with file-boundary and stream-end checks.
template <int kAbl, bool kC>
__device__ __forceinline__ void k1_word_slow(const K1Ctx& x, K1Stream& t, const v4u w, uint32_t S = 0) {
  const unsigned long long end = k1_end(x, t);
  // the current file's end from the stream state (lim = min(range end, file
  // end)): a file ending at or past the range end never ends inside it.  (The
  // offsets load this replaces cost every slow word an L2 round trip, four
  // per boundary line, for the whole wave.)  The next file's end is fetched
  // now if the file ends in this word, so its latency overlaps the bytes
  // before the boundary.
  unsigned long long fend = t.lim < end ? t.lim : ~0ull;
  unsigned long long fnext = fend < end && fend < t.p + 16 ? x.offsets[t.f + 2] : ~0ull;   // (fend < end: file t.f + 1 < nfiles)
  if (x.primary && ((w.x | w.y | w.z | w.w) & 0x80808080u) && t.p >= t.emit) k1_special(x, t, w, fend, end);
  // rolled (the slow path runs on boundary and last lines only): unrolled, its
  // 16 copies of the per-byte branches held ~450 scalar values live and the
  // kernel spilled SGPRs into VGPR lanes
#pragma unroll 1
  for (int k = 0; k < 16; ++k) {
    const unsigned long long q = t.p + k;
    if (q >= end) break;
    if (q >= fend) {
      if (kAbl & kAblBndNoFlush) t.kw0 = t.kw1 = 0;
      else if (kAbl & kAblBndRead) flush_kw(x.kwmask, x.kw_words, t.f, t.kw0, t.kw1);
      else flush_kw_blind(x.kwmask, x.kw_words, t.f, t.kw0, t.kw1);
      ++t.f;
      fend = fnext;
      while (q >= fend) { ++t.f; fend = x.offsets[t.f + 1]; }   // (empty files, files under 16 bytes)
      fnext = fend < end && fend < t.p + 16 ? x.offsets[t.f + 2] : ~0ull;   // a second boundary in this word
      t.s = x.s0;
      t.p12 = 0;
    }
    const uint32_t wk = (k & 8) ? ((k & 4) ? w.w : w.z) : ((k & 4) ? w.y : w.x);   // (no indexed array: scratch)
    const uint32_t b = (wk >> ((k & 3) * 8)) & 0xffu;
    if constexpr (kC) {
      const uint32_t c4 = x.cls[b];
      t.s = k1c_next(t.s, c4, __builtin_amdgcn_perm(0u, c4, 0u));
    } else {
      t.s = k1_step(x.next, t.s, (kAbl & kAblRootSkip) ? (x.cls[b] & 0xfeu) : x.cls[b]);
    }
    if (q >= t.emit) {
      t.nl += (b == 0x0au);
      if constexpr (kC) {
        if (t.s & 1u) k1_out_c(x, t, t.s, q);
      } else if (t.s >= x.first_out) {
        k1_out_v3(x, t, t.s, q, S);
      }
    }
    t.p12 = ((t.p12 << 8) & 0xff00u) | b;
  }
  t.p += 16;
  t.lim = min(end, fend);
}

// warm_bytes: a multiple of the kernel's line size (64 B; 128 B for the kAblLine64-off builds)
__device__ __forceinline__ void k1_init(const K1Ctx& x, K1Stream& t, unsigned long long c0, uint32_t warm_bytes) {
  t.emit = c0;
  t.p = c0 > warm_bytes ? c0 - warm_bytes : 0;   // c0 is a multiple of 128
  t.s = x.s0;
  t.p12 = 0;
  t.nl = 0;
  t.kw0 = t.kw1 = 0;
  t.end = min(c0 + x.chunk, x.total);
  t.cend = t.end;
  t.ci = 0;
  const unsigned long long end = t.end;
  if (c0 >= end) { t.p = t.lim = end; t.f = 0; return; }
  t.f = x.fidx ? file_of_idx(x.offsets, x.nfiles, x.fidx, t.p) : file_of(x.offsets, x.nfiles, t.p);
  t.lim = min(end, x.offsets[t.f + 1]);
}

// ==== K2 begin: K2 (from here to '==== K2 end') is outside K1's build hash
// (bench.py k1_build: the file up to here plus '==== K2 end' .. '==== host side')

// TSG_K2_STATS counters per rule: hits, gated hits, verify starts, verify
// bytes, the most verify bytes of one hit
constexpr uint32_t kK2Stat = 5;

// K2's per-anchor record (built on the host from AnchorInfo, RuleGpuInfo and
// the rule's verify / reverse DFA): everything a hit needs in four 16-byte
// loads issued together (rounds 1-4 walked anchor -> rule -> DFA records, three
// dependent L2 round trips before the first verify byte).
struct K2Anchor {
  uint32_t rule, min_len, max_len, dmin;
  uint32_t dmax, flags, kw_begin, kw_count;     // flags: mode | gate_on_gpu << 8 | always_gate << 9 | acc0 << 10 | racc0 << 11
  uint32_t verify_limit, v_next, v_cls, v_ncls_dead;   // ncls | dead << 16
  uint32_t r_next, r_cls, r_ncls_dead, kw0;     // reverse DFA (mode 4); kw0 = the rule's first keyword id
};
static_assert(sizeof(K2Anchor) == 64, "K2Anchor is four 16-byte loads");
// verify DFA transitions: next state | accepting << 15 (the accept flag rides
// with the state: one dependent load per byte instead of two)
constexpr uint32_t kVAcc = 0x8000u, kVState = 0x7fffu;

// The file of segment offset q from K1's per-chunk file (a lower bound: the
// file of the chunk's first byte or one before it), stepped forward; a chunk
// of many tiny files falls back to a binary search above the bound.
__device__ __forceinline__ uint32_t k2_file_of(const uint64_t* __restrict__ off, uint32_t nfiles,
                                               const uint32_t* __restrict__ chunk_file, uint32_t chunk,
                                               unsigned long long q) {
  uint32_t f = chunk_file[q / chunk];
  for (int k = 0; k < 4; ++k) {
    if (f >= nfiles || off[f + 1] > q) return f;
    ++f;
  }
  uint32_t lo = f, hi = nfiles;
  while (lo < hi) {
    const uint32_t m = (lo + hi + 1) >> 1;
    if (off[m] <= q) lo = m; else hi = m - 1;
  }
  f = lo;
  while (f < nfiles && off[f + 1] <= q) ++f;
  return f;
}

// K2: one thread per anchor hit.  The rule's keyword gate (K1's per-file
// bits), then the anchored relaxed verify DFA from every start the anchor's
// offset window allows (mode 0), or from every start a backward walk of the
// reverse DFA accepts (mode 4); mode 3 hits are presence candidates.
// Forward walks from up to kK2Walk starts run interleaved: their byte chains
// are independent, so one thread keeps kK2Walk dependent L2 round trips in
// flight instead of one.
constexpr int kK2Walk = 4;
// K2 builds: bit 0 = TSG_K2_STATS counters; probe library only (TSG_K2_ABL):
// bit 1 = per-wave wall-clock trace (results valid), bit 2 = no verify walks
// (results invalid: prices the setup of a hit)
constexpr int kK2Stats = 1, kK2Trace = 2, kK2NoWalk = 4;

template <int kK2>
__global__ __launch_bounds__(256) void tsg_k2_verify(
    const uint8_t* __restrict__ data, unsigned long long total, const uint64_t* __restrict__ offsets, uint32_t nfiles,
    const uint32_t* __restrict__ chunk_file, uint32_t chunk,
    const unsigned long long* __restrict__ hits, const uint32_t* __restrict__ block_hits, uint32_t region_cap,
    uint32_t nregions, uint32_t nsub_main, const unsigned long long* __restrict__ over_hits,
    const uint32_t* __restrict__ over_cnt, uint32_t over_cap,
    const K2Anchor* __restrict__ anchors, const uint32_t* __restrict__ rule_kw,
    const uint32_t* __restrict__ kwbits, uint32_t kw_words,
    const uint16_t* __restrict__ v_next, const uint8_t* __restrict__ v_cls,
    CandDev* __restrict__ cands, unsigned int* __restrict__ counters, uint32_t cand_cap,
    unsigned long long* __restrict__ k2s, uint32_t* __restrict__ trace) {
  constexpr bool kStats = (kK2 & kK2Stats) != 0;
  const uint32_t t_wave0 = (kK2 & kK2Trace) ? static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime()) : 0u;
  uint32_t tr_hits = 0, tr_bytes = 0;
  // The first nregions * nsub_main workgroups: workgroup (r, k) verifies K1
  // region r's hits k*256+tid, stride 256*nsub_main; the rest verify the
  // shared overflow pool the same way (one launch for both)
  uint32_t nhits, sub, nsub;
  const unsigned long long* __restrict__ rh;
  if (blockIdx.x < nregions * nsub_main) {
    const uint32_t r = blockIdx.x % nregions;
    nhits = min(block_hits[r], region_cap);
    rh = hits + static_cast<size_t>(r) * region_cap;
    sub = blockIdx.x / nregions;
    nsub = nsub_main;
  } else {
    nhits = min(*over_cnt, over_cap);
    rh = over_hits;
    sub = blockIdx.x - nregions * nsub_main;
    nsub = gridDim.x - nregions * nsub_main;
  }
  for (uint32_t i = sub * blockDim.x + threadIdx.x; i < nhits; i += nsub * blockDim.x) {
    const unsigned long long h = rh[i];
    const unsigned long long q = h >> 24;
    const K2Anchor an = anchors[h & 0xffffffu];
    if (kK2 & kK2Trace) ++tr_hits;
    const uint32_t f = k2_file_of(offsets, nfiles, chunk_file, chunk, q);
    const uint32_t mode = an.flags & 0xffu;
    if (kStats) atomicAdd(&k2s[kK2Stat * an.rule], 1ull);
    const unsigned long long fstart_u = offsets[f];
    auto emit = [&](unsigned long long start) {
      const unsigned int idx = atomicAdd(&counters[1], 1u);
      if (idx < cand_cap) {
        cands[idx].file = f;
        cands[idx].rule = an.rule;
        cands[idx].start = start;
      }
    };
    if (mode == 3) {
      // presence anchor of a rule evaluated in full on the host: the hit is
      // the candidate (any one per file suffices)
      emit(q - fstart_u);
      continue;
    }
    if (!(an.flags & 0x200u) && (an.flags & 0x100u)) {
      // keyword gate: any of the rule's keywords in the file (K1's bits)
      const uint32_t* kb = kwbits + static_cast<size_t>(f) * kw_words;
      uint32_t g = an.kw_count ? (kb[an.kw0 >> 5] >> (an.kw0 & 31)) & 1u : 0u;
      for (uint32_t k = 1; k < an.kw_count && !g; ++k) {
        const uint32_t id = rule_kw[an.kw_begin + k];
        g = (kb[id >> 5] >> (id & 31)) & 1u;
      }
      if (!g) continue;
    }
    if (kStats) atomicAdd(&k2s[kK2Stat * an.rule + 1], 1ull);
    const long long fstart = static_cast<long long>(fstart_u);
    const long long fend = static_cast<long long>(offsets[f + 1]);
    unsigned long long hit_bytes = 0;
    const uint16_t* nx = v_next + an.v_next;
    const uint8_t* cl = v_cls + an.v_cls;
    const uint32_t ncls = an.v_ncls_dead & 0xffffu, dead = an.v_ncls_dead >> 16;
    const bool acc0 = (an.flags & 0x400u) != 0;
    // up to kK2Walk anchored verify walks from starts s0 .. s0+n-1 (ascending),
    // interleaved; *res bit j: a prefix of the text from start j lies in the
    // rule's relaxed language (or the walk gave up alive at its byte limit:
    // conservative)
    auto verify_n = [&](const long long* st0, int n) -> uint32_t {
      uint32_t res = 0, live = 0;
      if (kK2 & kK2NoWalk) return 0u;
      // positions as 32-bit offsets from wb, the 16-byte boundary at or below
      // the first start (a walk spans at most verify_limit + 3 bytes)
      const long long wb = st0[0] & ~15ll;
      const uint32_t ofend = static_cast<uint32_t>(min(fend - wb, 0x7fffffffll));
      uint32_t stt[kK2Walk], o[kK2Walk], olim[kK2Walk];
#pragma unroll
      for (int j = 0; j < kK2Walk; ++j) {
        stt[j] = 0;
        o[j] = j < n ? static_cast<uint32_t>(st0[j] - wb) : 0u;
        olim[j] = j < n ? min(ofend, o[j] + an.verify_limit) : 0u;
        if (j < n) {
          if (acc0) res |= 1u << j;
          else if (o[j] < olim[j]) live |= 1u << j;
          else if (olim[j] < ofend && dead != 0) res |= 1u << j;   // a zero byte limit before the file end: gave up alive
        }
      }
      // (round 5 measured a class window -- the classes of the 32 text bytes
      // from wb looked up together into an LDS slot, one dependent load per
      // step instead of three -- and a walk budget with a deferred pass for
      // long-walking lanes: both slower, profiles/r5k_*, r5l_*, r5n_*)
      while (live) {
        uint32_t b[kK2Walk];
#pragma unroll
        for (int j = 0; j < kK2Walk; ++j) b[j] = (live >> j) & 1u ? data[wb + o[j]] : 0u;
        uint32_t c[kK2Walk];
#pragma unroll
        for (int j = 0; j < kK2Walk; ++j) c[j] = cl[b[j]];
#pragma unroll
        for (int j = 0; j < kK2Walk; ++j) {
          if (!((live >> j) & 1u)) continue;
          const uint32_t e = nx[stt[j] * ncls + c[j]];
          stt[j] = e & kVState;
          ++o[j];
          if (kStats) hit_bytes += 1;
          if (kK2 & kK2Trace) ++tr_bytes;
          if (e & kVAcc) { res |= 1u << j; live &= ~(1u << j); }
          else if (stt[j] == dead) live &= ~(1u << j);
          else if (o[j] >= olim[j]) {
            live &= ~(1u << j);
            if (o[j] < ofend) res |= 1u << j;           // gave up alive at the byte limit: conservative
          }
        }
      }
      if (kStats) {
        atomicAdd(&k2s[kK2Stat * an.rule + 2], static_cast<unsigned long long>(n));
      }
      return res;
    };
    if (mode == 4) {
      // reverse-anchored: walk the reverse DFA backwards from the hit's last
      // byte; every accepting position may start a match and is verified
      // forwards.  A walk still alive after kRevLimit bytes gives up: the
      // host evaluates the rule on the whole file (kFullScanStart).
      const uint16_t* rnx = v_next + an.r_next;
      const uint8_t* rcl = v_cls + an.r_cls;
      const uint32_t rncls = an.r_ncls_dead & 0xffffu, rdead = an.r_ncls_dead >> 16;
      uint32_t st = 0;
      for (long long pp = static_cast<long long>(q); pp >= fstart; --pp) {
        if (static_cast<long long>(q) - pp >= static_cast<long long>(kRevLimit)) { emit(kFullScanStart); break; }
        const uint32_t e = rnx[st * rncls + rcl[data[pp]]];
        st = e & kVState;
        if (kStats) ++hit_bytes;
        if (st == rdead) break;
        if (e & kVAcc) {
          const long long s1 = pp;
          if (verify_n(&s1, 1) & 1u) emit(static_cast<unsigned long long>(pp - fstart));
        }
      }
      if (kStats) {
        atomicAdd(&k2s[kK2Stat * an.rule + 3], hit_bytes);
        atomicMax(&k2s[kK2Stat * an.rule + 4], hit_bytes);
      }
      continue;
    }
    long long hi = static_cast<long long>(q) + 1 - an.min_len - an.dmin;
    long long lo = static_cast<long long>(q) + 1 - an.max_len - an.dmax;
    if (lo < fstart) lo = fstart;
    for (long long s0 = lo; s0 <= hi; s0 += kK2Walk) {
      long long st0[kK2Walk];
      const int n = static_cast<int>(min(static_cast<long long>(kK2Walk), hi - s0 + 1));
#pragma unroll
      for (int j = 0; j < kK2Walk; ++j) st0[j] = s0 + j;
      const uint32_t res = verify_n(st0, n);
      for (int j = 0; j < n; ++j)
        if ((res >> j) & 1u) emit(static_cast<unsigned long long>(s0 + j - fstart));
    }
    if (kStats) {
      atomicAdd(&k2s[kK2Stat * an.rule + 3], hit_bytes);
      atomicMax(&k2s[kK2Stat * an.rule + 4], hit_bytes);
    }
  }
  if (kK2 & kK2Trace) {
    // per wave: [start, end, hits (sum over lanes), walk bytes (sum), most hits of a lane, most bytes of a lane]
    uint32_t sh = tr_hits, sb = tr_bytes, mh = tr_hits, mb = tr_bytes;
    for (int o = 32; o > 0; o >>= 1) {
      sh += __shfl_xor(sh, o);
      sb += __shfl_xor(sb, o);
      mh = max(mh, static_cast<uint32_t>(__shfl_xor(mh, o)));
      mb = max(mb, static_cast<uint32_t>(__shfl_xor(mb, o)));
    }
    if ((threadIdx.x & 63u) == 0) {
      uint32_t* r = trace + 8 * (static_cast<size_t>(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64);
      r[0] = t_wave0;
      r[1] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
      r[2] = sh; r[3] = sb; r[4] = mh; r[5] = mb; r[6] = blockIdx.x; r[7] = 0;
    }
  }
}

// ==== K2 end: from here to '==== host side' is K1 again (in k1_build)

// K1 v3: the same pass, built around the per-byte cost.
//  * LDS layout [class map (256 B) | scan table | output meta | output list |
//    per-wave hit buffers | counters]: the class map and the table sit at
//    compile-time offsets below 64 KiB, so a class lookup is one ds_read_u8
//    addressed by the byte itself and a transition one v_lshl_add + one
//    ds_read_u16 with an immediate offset;
//  * 128-byte lines are double-buffered in registers: the next line's loads
//    are in flight while this one is walked;
//  * newlines are counted with one popcount per dword (32 - popc of the
//    zero-byte mask word);
//  * output positions of a word are found from one max over its 16 states,
//    then handled through a position mask, so each word carries one copy of
//    the output code;
//  * wave work items come from one global counter per launch (no static
//    per-workgroup ranges, no tail of idle CUs).
// kAbl (measurement only, results are wrong with any bit set except
// kAblTemporal): drop a part of the per-byte work to price it.
constexpr int kAblNoNl = 1, kAblNoOut = 2, kAblNoCls = 4, kAblNoSpecial = 8, kAblTemporal = 16, kAblLoadOnly = 32;
// layout bits (results stay valid): 64-byte lines instead of 128; word loop
// rolled (register-indexed) instead of unrolled
constexpr int kAblLine64 = 64, kAblRolled = 128, kAblDefer = 256;
// measurement only: every line load reads the batch's first 1 MiB instead
// (L2-resident), pricing the per-byte work without HBM
constexpr int kAblNoLoad = 512;
// measurement only: transitions addressed by pointer arithmetic on the
// dynamic-LDS pointer (two VALU per byte) instead of the integer LDS address
constexpr int kAblPtrAddr = 1024;
// layout bit (results valid): no register double buffer -- a line's loads are
// issued together when the line starts (a 128-byte line is then fetched in one
// burst instead of two halves microseconds apart)
constexpr int kAblSingle = 2048;
// layout bits (results valid) for lines holding a file boundary: the words
// wholly inside the current file take the fast word step (only the word with
// the boundary runs the byte loop); and reloading such a line's words one by
// one from memory, dropping the register prefetch (rounds 1-3)
constexpr int kAblBoundaryFastWords = 4096, kAblBoundaryReload = 8192;
// Deferred outputs (kAblDefer): a lane parks each output position of its
// fast lines as (offset from the chunk start << 16 | state) in its own slots
// of a global buffer (L2-resident) and handles them when its file or chunk
// ends, every lane at once, instead of the wave stopping at each position
// where any lane has one.
constexpr uint32_t kOutSlots = 8;
struct OutBuf { uint32_t* p; uint32_t stride, n; };

template <int kAbl>
__device__ __forceinline__ v4u k1_load(const uint8_t* data, unsigned long long off) {
  if (kAbl & kAblNoLoad) off &= 0xfffffull;   // the batch holds >= 1 MiB in these runs (checked on the host)
  const uint8_t* p = data + off;
  if (kAbl & kAblTemporal) return *reinterpret_cast<const v4u*>(p);
  return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
}

// Does a U+0130 / U+017F / U+212A encoding end inside the 128-byte line at p
// (p12: the two bytes before it)?  Out of line: only lines with a byte >= 0x80
// get here.  The fast path's line lies in one file, which is flagged.
__device__ __noinline__ bool k1_line_special(const uint8_t* __restrict__ p, uint32_t p12, uint32_t n) {
  uint32_t a = p12 & 0xffu, bb = p12 >> 8;
  bool hit = false;
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t b = p[k];
    hit |= (b == 0xB0u && a == 0xC4u) || (b == 0xBFu && a == 0xC5u) || (b == 0xAAu && a == 0x84u && bb == 0xE2u);
    bb = a;
    a = b;
  }
  return hit;
}

// The same test with the line's words loaded together (round 6; the call
// site's line is 16-byte aligned): one L2 round trip per 16 bytes, the next
// word's load in flight, instead of one dependent byte load per byte.  The byte loop above took ~20-35 us per line under a
// loaded memory system with the whole wave waiting: in a 17 MB file of
// config-2-like text with a stray lead byte every ~40 KB (synth's 0.05% of
// files with invalid UTF-8) every 8 KiB item ran ~450 us longer, and such a
// file's items set the launch's end (2.5 GB launch 1.02 ms, the slowest
// items 0.9-1.0 ms against a median of 0.56; profiles/r7u_*).  Out of line:
// the test inlined on the line's registers pushed K1 to 128 VGPRs with 32
// spilled (4 GB launch 1.16 -> 2.07 ms, profiles/r7v_*).  Per dword w (pw: the
// dword before it) a byte ends a sequence when it and its one or two
// predecessors all match, i.e. when the OR of their XORs with the sequence
// bytes is a zero byte: funnel shifts give the predecessors, and one
// any-zero-byte test per sequence (exact as an any-byte test) decides.
__device__ __forceinline__ uint32_t k1_any_zero(uint32_t x) { return (x - 0x01010101u) & ~x & 0x80808080u; }
__device__ __noinline__ bool k1_line_special_words(const uint8_t* __restrict__ p, uint32_t p12, uint32_t n) {
  uint32_t pw = ((p12 & 0xffu) << 24) | ((p12 & 0xff00u) << 8);   // byte 3: the byte before the line, byte 2: the one before that
  uint32_t hit = 0;
  // one word in flight ahead of the one tested, rolled: a callee with many
  // live VGPRs makes the call site save K1's registers (8 words loaded at once
  // left K1 with 32 VGPRs spilled)
  v4u nx = *reinterpret_cast<const v4u*>(p);
#pragma unroll 1
  for (uint32_t o = 0; o < n; o += 16) {
    const v4u cw = nx;
    if (o + 16 < n) nx = *reinterpret_cast<const v4u*>(p + o + 16);
    const uint32_t d[4] = {cw.x, cw.y, cw.z, cw.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t w = d[j];
      const uint32_t p1 = __builtin_amdgcn_alignbit(w, pw, 24);   // byte k: byte k - 1
      const uint32_t p2 = __builtin_amdgcn_alignbit(w, pw, 16);   // byte k: byte k - 2
      hit |= k1_any_zero((w ^ 0xB0B0B0B0u) | (p1 ^ 0xC4C4C4C4u))                          // U+0130 C4 B0
           | k1_any_zero((w ^ 0xBFBFBFBFu) | (p1 ^ 0xC5C5C5C5u))                          // U+017F C5 BF
           | k1_any_zero((w ^ 0xAAAAAAAAu) | (p1 ^ 0x84848484u) | (p2 ^ 0xE2E2E2E2u));   // U+212A E2 84 AA
      pw = w;
    }
  }
  return hit != 0;
}

// Can a line (plus the two bytes before it, p12) hold one of those
// sequences at all: does it contain a lead byte C4 / C5 / E2?  Exact as an
// any-byte test (a borrow can only flag bytes above a zero byte), run on the
// line's registers before the out-of-line byte check, which re-reads the line
// from memory: text with other non-ASCII letters (C3 xx, D0 xx, CJK) rarely
// gets past it.  Small files with such text ran K1 15% slower with the byte
// check on every non-ASCII line (probe variant 472 vs 464).
__device__ __forceinline__ uint32_t k1_has_lead(uint32_t w) {
  const uint32_t a = (w & 0xFEFEFEFEu) ^ 0xC4C4C4C4u;   // C4 or C5 -> zero byte
  const uint32_t b = w ^ 0xE2E2E2E2u;
  return (((a - 0x01010101u) & ~a) | ((b - 0x01010101u) & ~b)) & 0x80808080u;
}

// a parked output: (offset from the range start << 16) | state (K1: row
// offset; K1c: DESC address)
template <bool kC>
__device__ __forceinline__ void k1_drain(const K1Ctx& x, K1Stream& t, OutBuf& ob, uint32_t S) {
  for (uint32_t i = 0; i < ob.n; ++i) {
    const uint32_t e = ob.p[i * ob.stride];
    if constexpr (kC) k1_out_c(x, t, e & 0xfff0u, t.emit + (e >> 16));
    else k1_out_v3(x, t, e & 0xffffu, t.emit + (e >> 16), S);
  }
  ob.n = 0;
}

template <int kAbl, bool kC>
__device__ __forceinline__ void k1_word_v3(const K1Ctx& x, K1Stream& t, OutBuf& ob, const uint8_t* smem, uint32_t S,
                                           uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  constexpr uint32_t kTabOff = 256;
  const bool emit = t.p >= t.emit;
  if (kAbl & kAblLoadOnly) {            // the loads kept live through kw1 (discarded at the end)
    t.kw1 += w0 ^ w1 ^ w2 ^ w3;
    t.p += 16;
    return;
  }
  const uint32_t w[4] = {w0, w1, w2, w3};
  uint32_t c2[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t b = (w[k >> 2] >> ((k & 3) * 8)) & 0xffu;
    c2[k] = (kAbl & kAblNoCls) ? ((b & 31u) << 1) : static_cast<uint32_t>(smem[b]);   // NoCls: nclasses >= 32
  }
  uint32_t st[16];
  uint32_t s = t.s;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if constexpr (kC) s = k1c_next(s, c2[k], __builtin_amdgcn_perm(0u, c2[k], 0u));   // K1c: class * 4 in every byte
    else if (kAbl & kAblPtrAddr) s = *reinterpret_cast<const uint16_t*>(smem + kTabOff + (s << 2) + c2[k]);
    else if (kAbl & kAblRootSkip) {
      // (s | flag ^ 1) == 0: at the start state (row offset 0) on a self-loop class
      if ((s | ((c2[k] & 1u) ^ 1u)) != 0u) s = k1_lds16((s << 2) + (c2[k] & 0xfeu) + kTabOff);
    }
    else s = k1_lds16((s << 2) + c2[k] + kTabOff);
    st[k] = s;
  }
  t.s = s;
  if (emit) {
    if (!(kAbl & kAblNoNl)) {
      uint32_t u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t xx = w[j] ^ 0x0a0a0a0au;
        u[j] = ((xx & 0x7f7f7f7fu) + 0x7f7f7f7fu) | xx | 0x7f7f7f7fu;   // bit 7 of a byte: not '\n'
      }
      t.nl += 128u - (__popc(u[0]) + __popc(u[1]) + __popc(u[2]) + __popc(u[3]));
    }
    if (!(kAbl & kAblNoOut)) {
      // outputs: one max per 4 positions decides (wave-wide) whether to look
      // at them one by one; each output position costs one LDS round trip
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool any = kC ? ((st[4 * j] | st[4 * j + 1] | st[4 * j + 2] | st[4 * j + 3]) & 1u) != 0
                            : max(max(st[4 * j], st[4 * j + 1]), max(st[4 * j + 2], st[4 * j + 3])) >= x.first_out;
        if (any) {
#pragma unroll
          for (int k = 4 * j; k < 4 * j + 4; ++k) {
            if (kC ? (st[k] & 1u) != 0 : st[k] >= x.first_out) {
              if ((kAbl & kAblDefer) && ob.n < kOutSlots) {
                const uint32_t tag = kC ? (st[k] & 0xfff0u) : st[k];
                ob.p[ob.n * ob.stride] = (static_cast<uint32_t>(t.p + k - t.emit) << 16) | tag;
                ++ob.n;
              } else if constexpr (kC) {
                k1_out_c(x, t, st[k], t.p + k);
              } else {
                k1_out_v3(x, t, st[k], t.p + k, S);
              }
            }
          }
        }
      }
    }
  }
  t.p12 = (w3 >> 24) | ((w3 >> 8) & 0xff00u);
  t.p += 16;
}

// K1c's 16-byte word: two halves of 8 bytes (8 class reads, then the 8
// dependent steps, then their outputs), so the two-read step's registers fit
// the 128-VGPR budget of 1024-thread workgroups without spilling.
// measurement only (invalid results): K1c's step with the row read alone
// (no record), or with both reads but no exception test (their values
// folded by two VALU): prices the record read and the select chain
constexpr int kAblCRowOnly = 16384, kAblCNoSelect = 32768;
template <int kAbl>
__device__ __forceinline__ uint32_t k1c_step_abl(uint32_t s, uint32_t c4) {
  if constexpr ((kAbl & kAblCRowOnly) != 0) {
    return k1_lds32(((s >> 16) << 2) + c4);
  } else if constexpr ((kAbl & kAblCNoSelect) != 0) {
    const uint32_t f = k1_lds32(((s >> 16) << 2) + c4);
    const v4u d = k1_lds128(s & 0xfff0u);
    return f ^ (d.y & 0x10u);
  } else {
    return k1c_next(s, c4, __builtin_amdgcn_perm(0u, c4, 0u));   // c4 in every byte
  }
}

template <int kAbl>
__device__ __forceinline__ void k1_word_c(const K1Ctx& x, K1Stream& t, OutBuf& ob, const uint8_t* smem,
                                          uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  const bool emit = t.p >= t.emit;
  const uint32_t w[4] = {w0, w1, w2, w3};
  uint32_t s = t.s;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t c4[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c4[k] = smem[(w[2 * h + (k >> 2)] >> ((k & 3) * 8)) & 0xffu];
    uint32_t st[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s = k1c_step_abl<kAbl>(s, c4[k]);
      st[k] = s;
    }
    if (emit) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if ((st[4 * j] | st[4 * j + 1] | st[4 * j + 2] | st[4 * j + 3]) & 1u) {
#pragma unroll
          for (int k = 4 * j; k < 4 * j + 4; ++k) {
            if (st[k] & 1u) {
              const unsigned long long q = t.p + 8 * h + k;
              if (ob.n < kOutSlots) {
                ob.p[ob.n * ob.stride] = (static_cast<uint32_t>(q - t.emit) << 16) | (st[k] & 0xfff0u);
                ++ob.n;
              } else {
                k1_out_c(x, t, st[k], q);
              }
            }
          }
        }
      }
    }
  }
  t.s = s;
  if (emit) {
    uint32_t u[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t xx = w[j] ^ 0x0a0a0a0au;
      u[j] = ((xx & 0x7f7f7f7fu) + 0x7f7f7f7fu) | xx | 0x7f7f7f7fu;   // bit 7 of a byte: not '\n'
    }
    t.nl += 128u - (__popc(u[0]) + __popc(u[1]) + __popc(u[2]) + __popc(u[3]));
  }
  t.p12 = (w3 >> 24) | ((w3 >> 8) & 0xff00u);
  t.p += 16;
}

template <int kThreads, int kAbl, bool kC>
__global__ __launch_bounds__(kThreads) void tsg_k1_scan_v3(
    const uint8_t* __restrict__ data, unsigned long long total,
    const uint64_t* __restrict__ offsets, uint32_t nfiles,
    const uint16_t* __restrict__ g_next, const uint8_t* __restrict__ g_cls,
    uint32_t nclasses, uint32_t table_words16, uint32_t first_out,
    const OutMeta* __restrict__ g_meta, uint32_t wave_hits, const uint32_t* __restrict__ g_list, uint32_t nlist,
    uint32_t nkw, uint32_t warm_lines, uint32_t chunk, unsigned long long nchunks,
    uint32_t* __restrict__ kwbits, uint32_t kw_words, uint32_t kw_base, uint32_t primary,
    unsigned long long* __restrict__ hits, uint32_t* __restrict__ block_hits, uint32_t region_cap,
    unsigned long long* __restrict__ over, uint32_t* __restrict__ over_cnt, uint32_t over_cap,
    uint16_t* __restrict__ nl_count, uint32_t* __restrict__ chunk_file, uint32_t* __restrict__ fflags,
    uint32_t* __restrict__ item_ctr, uint32_t* __restrict__ obuf, uint32_t tail_rounds,
    const uint32_t* __restrict__ fidx) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr uint32_t kWaves = kThreads / 64;
  constexpr uint32_t kTabOff = 256;
  // kAblTrace: [4 per workgroup: entry, table loaded, exit, hw id][kTraceItemWords per item: start, end,
  // kU << 24 | wg << 8 | wave, range set up (file found), line loop done, outputs drained + keyword bits flushed]
  uint32_t* const trc = obuf + static_cast<size_t>(gridDim.x) * kThreads * kOutSlots;
  if ((kAbl & kAblTrace) && threadIdx.x == 0) {
    trc[4 * blockIdx.x] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
    trc[4 * blockIdx.x + 3] = __smid();
  }
  if (!(kAbl & kAblPtrAddr) && !k1_lds_base_ok(smem)) {   // the integer LDS addresses assume a zero base
    if (threadIdx.x == 0) atomicOr(over_cnt + 1, 1u);
    return;
  }
  const uint32_t padded = (table_words16 * 2 + 15) & ~15u;
  const uint32_t meta_off = kTabOff + padded;
  const uint32_t list_off = meta_off;            // output metadata is inline in the table rows (K1c: in global memory)
  const uint32_t hits_off = (list_off + (kC ? 0u : nlist * 4) + 15) & ~15u;
  uint32_t S = (nclasses + 2) & ~1u;             // k1_row_stride(nclasses): the silent-row stride
  if (((S / 2) & 1u) == 0) S += 2;
  uint32_t* s_hits = reinterpret_cast<uint32_t*>(smem + hits_off);
  uint32_t* s_hitcnt = s_hits + kWaves * wave_hits;
  uint32_t* s_block = s_hitcnt + kMaxWaves;      // [0] region fill count
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_block[0] = 0;
  {
    const uint4* src = reinterpret_cast<const uint4*>(g_next);
    uint4* dst = reinterpret_cast<uint4*>(smem + kTabOff);
    for (uint32_t i = threadIdx.x; i < padded / 16; i += blockDim.x) dst[i] = src[i];
    for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
      uint32_t c = g_cls[i];
      if (!kC && (kAbl & kAblRootSkip) && g_next[c >> 1] == 0) c |= 1u;   // row 0 = the start state's row
      smem[i] = static_cast<uint8_t>(c);
    }
    if (!kC) {
      uint32_t* s_list = reinterpret_cast<uint32_t*>(smem + list_off);
      for (uint32_t i = threadIdx.x; i < nlist; i += blockDim.x) s_list[i] = g_list[i];
    }
  }
  K1Ctx x;
  x.data = data; x.total = total; x.chunk = chunk;
  x.offsets = offsets; x.nfiles = nfiles; x.fidx = fidx;
  x.next = reinterpret_cast<const uint16_t*>(smem + kTabOff);
  x.cls = smem;
  x.first_out = first_out; x.nclasses = nclasses; x.wave_hits = wave_hits;
  x.meta = kC ? g_meta : nullptr;
  x.list = kC ? g_list : reinterpret_cast<const uint32_t*>(smem + list_off);
  x.s0 = kC ? first_out : 0u;                    // K1c: first_out carries the start state's packed value
  x.nkw = nkw;
  x.kwbits = kwbits; x.kwmask = kwbits + kw_base / 32; x.kw_words = kw_words; x.primary = primary != 0;
  x.hits = hits + static_cast<size_t>(blockIdx.x) * region_cap; x.region_cap = region_cap; x.b_hitcnt = s_block;
  x.over = over; x.over_cnt = over_cnt; x.over_cap = over_cap;
  x.w_hits = s_hits + wid * wave_hits; x.w_hitcnt = s_hitcnt + wid; x.fflags = fflags;
  __syncthreads();
  // Guided work schedule.  A wave item gives each of its 64 lanes a range of
  // kU consecutive chunks, walked as one stream (one warm-up) that stores the
  // '\n' count of every chunk it crosses.  Items come from one counter in
  // decreasing range size: kU = 4 for the bulk, then `tail_rounds` grid-wide
  // rounds of kU = 2 and as many of kU = 1, so the waves that take the last
  // items finish after a short item and the launch has no long tail
  // (measured r2u, 4 GB: 1.29 ms without the short rounds, 1.21 with one
  // round each, 1.24 / 1.27 with two / four).  With bit 8 of tail_rounds
  // (round 6, launches of >= 2 GiB at half the chunk) the bulk is kU = 8 and
  // kU = 4 gets `tail_rounds` rounds too: the same bulk ranges, the last
  // round's ranges half as long.
  const uint32_t rounds = tail_rounds & 0xffu;
  const bool top8 = (tail_rounds & 0x100u) != 0;
  const unsigned long long W = static_cast<unsigned long long>(gridDim.x) * kWaves;
  const unsigned long long n1 = min(nchunks, W * 64 * rounds);
  const unsigned long long n2 = min(nchunks - n1, W * 128 * rounds);
  const unsigned long long n4 = top8 ? min(nchunks - n1 - n2, W * 256 * rounds) : nchunks - n1 - n2;
  const unsigned long long n8 = nchunks - n1 - n2 - n4;
  const unsigned long long i8 = (n8 + 511) / 512, i4 = (n4 + 255) / 256, i2 = (n2 + 127) / 128;
  const unsigned long long nitems = i8 + i4 + i2 + (n1 + 63) / 64;
  if ((kAbl & kAblTrace) && threadIdx.x == 0) trc[4 * blockIdx.x + 1] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
  bool first = !(kAbl & kAblAtomicFirst);
  // the next item from the counters (lane 0)
  auto take = [&]() -> unsigned long long {
    if (!(kAbl & (kAblOneCounter | kAblAtomicFirst))) {
      const uint32_t xc = blockIdx.x & 7u;
      return W + xc + 8ull * atomicAdd(item_ctr + 32 * xc, 1u);
    }
    return atomicAdd(item_ctr, 1u) + ((kAbl & kAblAtomicFirst) ? 0ull : W);
  };
  for (;;) {
    unsigned long long item = 0;
    const uint32_t t_item = (kAbl & kAblTrace) ? static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime()) : 0u;
    uint32_t t_setup = 0, t_loop = 0, t_kw = 0;    // (kAblTrace)
    if (first) {
      // the first round of items: wave w of the grid takes item w (no atomic);
      // the counter then hands out items W, W + 1, ...
      item = static_cast<unsigned long long>(blockIdx.x) * kWaves + wid;
      if (lane == 0) *x.w_hitcnt = 0;
      first = false;
    } else {
      if (lane == 0) {
        item = take();
        *x.w_hitcnt = 0;
      }
      item = __shfl(item, 0);
    }
    if (item >= nitems) break;                                 // wave-uniform exit
    __builtin_amdgcn_wave_barrier();
    unsigned long long c0, rend;
    uint32_t kU;
    if (item < i8) { kU = 8; c0 = item * 512; rend = n8; }
    else if (item < i8 + i4) { kU = 4; c0 = n8 + (item - i8) * 256; rend = n8 + n4; }
    else if (item < i8 + i4 + i2) { kU = 2; c0 = n8 + n4 + (item - i8 - i4) * 128; rend = n8 + n4 + n2; }
    else { kU = 1; c0 = n8 + n4 + n2 + (item - i8 - i4 - i2) * 64; rend = nchunks; }
    x.item_base = c0 * static_cast<unsigned long long>(chunk);   // hit offsets < 64 * kU chunks (k1_max_chunk(kU), host-checked)
    const unsigned long long c = c0 + lane * kU;                 // the lane's first chunk
    if (c < rend) {
      K1Stream t;
      // v3 warms up over whole lines of its own size (warm_lines counts them)
      k1_init(x, t, min(c * chunk, total), warm_lines * ((kAbl & kAblLine64) ? 64u : 128u));
      t.end = min(min(c + kU, rend) * chunk, total);
      t.cend = min(t.emit + chunk, t.end);
      t.ci = c;
      if (x.primary) chunk_file[c] = t.f;            // K2's file lookup: a file at or before the chunk's first byte
      if (t.p < t.end) t.lim = min(t.end, x.offsets[t.f + 1]);
      OutBuf ob{obuf + blockIdx.x * kThreads + threadIdx.x, gridDim.x * kThreads, 0};
      if (kAbl & kAblTrace) t_setup = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
      constexpr int kW = (kAbl & kAblLine64) ? 4 : 8;     // words per line
      constexpr uint32_t kL = kW * 16;
      v4u cur[kW], nxt[kW];
      bool have = false;
      for (;;) {
        if (!(t.p < t.lim || t.p < k1_end(x, t))) break;
        if (t.p >= t.cend && t.cend < t.end) {                // a chunk of the range is done: store its
          if (x.primary) nl_count[t.ci] = static_cast<uint16_t>(t.nl);   // count before any byte of the next
          t.nl = 0;
          ++t.ci;
          if (x.primary) chunk_file[t.ci] = t.f;        // (a lower bound of the chunk's first file: K2)
          t.cend = min(t.cend + chunk, t.end);
        }
        // a whole line inside the lane's range is loaded (and the next one
        // prefetched) whatever file boundaries it holds; lines wholly inside
        // the current file take the fast word steps
        const bool reload = (kAbl & kAblBoundaryReload) != 0;
        const bool in_file = t.p + kL <= t.lim;
        if (reload ? in_file : t.p + kL <= k1_end(x, t)) {
          if (!have) {
#pragma unroll
            for (int i = 0; i < kW; ++i) cur[i] = k1_load<kAbl>(data, t.p + 16 * i);
          }
          have = !(kAbl & kAblSingle) && t.p + 2 * kL <= (reload ? t.lim : k1_end(x, t));
          if (have) {
#pragma unroll
            for (int i = 0; i < kW; ++i) nxt[i] = k1_load<kAbl>(data, t.p + kL + 16 * i);
          }
          if (in_file) {
            if (!(kAbl & (kAblNoSpecial | kAblLoadOnly)) && x.primary) {
              uint32_t hb = 0;
#pragma unroll
              for (int i = 0; i < kW; ++i) hb |= cur[i].x | cur[i].y | cur[i].z | cur[i].w;
              if (hb & 0x80808080u) {
                uint32_t lead = k1_has_lead(t.p12);
#pragma unroll
                for (int i = 0; i < kW; ++i)
                  lead |= k1_has_lead(cur[i].x) | k1_has_lead(cur[i].y) | k1_has_lead(cur[i].z) | k1_has_lead(cur[i].w);
                if (lead && ((kAbl & kAblSpecialMem) ? k1_line_special(data + t.p, t.p12, kL)
                                                     : k1_line_special_words(data + t.p, t.p12, kL)))
                  atomicOr(&x.fflags[t.f], 1u);
              }
            }
            if (kAbl & kAblRolled) {
              // one copy of the word body: the uniform word index selects
              // cur[i] by register indexing
#pragma unroll 1
              for (int i = 0; i < kW; ++i) {
                if constexpr (kC) k1_word_c<kAbl>(x, t, ob, smem, cur[i].x, cur[i].y, cur[i].z, cur[i].w);
                else k1_word_v3<kAbl, kC>(x, t, ob, smem, S, cur[i].x, cur[i].y, cur[i].z, cur[i].w);
              }
            } else {
#pragma unroll
              for (int i = 0; i < kW; ++i) {
                if constexpr (kC) k1_word_c<kAbl>(x, t, ob, smem, cur[i].x, cur[i].y, cur[i].z, cur[i].w);
                else k1_word_v3<kAbl, kC>(x, t, ob, smem, S, cur[i].x, cur[i].y, cur[i].z, cur[i].w);
              }
            }
          } else {
            // a line holding a file boundary: its words (already in
            // registers) through the byte loop, which switches files; parked
            // outputs belong to file t.f, so they are handled first.  A
            // boundary every ~21 KB (image layers) used to reload the line's
            // words one by one and restart the prefetch: four exposed memory
            // latencies per boundary for the whole wave.
            if (kAbl & kAblDefer) k1_drain<kC>(x, t, ob, S);
#pragma unroll 1
            for (int i = 0; i < kW; ++i) {
              if (t.p >= k1_end(x, t)) break;
              if (t.p >= t.cend && t.cend < t.end) {            // chunk ends are word-aligned
                if (x.primary) nl_count[t.ci] = static_cast<uint16_t>(t.nl);
                t.nl = 0;
                ++t.ci;
                if (x.primary) chunk_file[t.ci] = t.f;        // (a lower bound of the chunk's first file: K2)
                t.cend = min(t.cend + chunk, t.end);
              }
              // (the word by selects, not by an indexed register array: the
              // rolled loop would put cur[] in scratch)
              v4u cw = cur[0];
#pragma unroll
              for (int j = 1; j < kW; ++j) cw = i == j ? cur[j] : cw;
              if ((kAbl & kAblDefer) && (kAbl & kAblBoundaryFastWords) && t.p + 16 <= t.lim) {
                if (x.primary && ((cw.x | cw.y | cw.z | cw.w) & 0x80808080u) && t.p >= t.emit)
                  k1_special(x, t, cw, x.offsets[t.f + 1], k1_end(x, t));
                if constexpr (kC) k1_word_c<kAbl>(x, t, ob, smem, cw.x, cw.y, cw.z, cw.w);
                else k1_word_v3<kAbl, kC>(x, t, ob, smem, S, cw.x, cw.y, cw.z, cw.w);
              } else {
                if (kAbl & kAblDefer) k1_drain<kC>(x, t, ob, S);
                k1_word_slow<kAbl, kC>(x, t, cw, S);
              }
            }
          }
          if (have) {
#pragma unroll
            for (int i = 0; i < kW; ++i) cur[i] = nxt[i];
          }
        } else {
          // the range's last, partial line (or, with kAblBoundaryReload, any
          // line holding a file boundary): word by word from memory
          have = false;
          if (kAbl & kAblDefer) k1_drain<kC>(x, t, ob, S);     // parked outputs belong to file t.f
#pragma unroll 1
          for (int i = 0; i < kW && t.p < k1_end(x, t); ++i) {
            if (t.p >= t.cend && t.cend < t.end) {            // chunk ends are word-aligned
              if (x.primary) nl_count[t.ci] = static_cast<uint16_t>(t.nl);
              t.nl = 0;
              ++t.ci;
              if (x.primary) chunk_file[t.ci] = t.f;        // (a lower bound of the chunk's first file: K2)
              t.cend = min(t.cend + chunk, t.end);
            }
            const v4u v = *reinterpret_cast<const v4u*>(data + t.p);
            if ((kAbl & kAblDefer) && (kAbl & kAblBoundaryFastWords) && t.p + 16 <= t.lim) {
              if (x.primary && ((v.x | v.y | v.z | v.w) & 0x80808080u) && t.p >= t.emit)
                k1_special(x, t, v, x.offsets[t.f + 1], k1_end(x, t));
              if constexpr (kC) k1_word_c<kAbl>(x, t, ob, smem, v.x, v.y, v.z, v.w);
              else k1_word_v3<kAbl, kC>(x, t, ob, smem, S, v.x, v.y, v.z, v.w);
            } else {
              if (kAbl & kAblDefer) k1_drain<kC>(x, t, ob, S);   // before the word that may change the file
              k1_word_slow<kAbl, kC>(x, t, v, S);
            }
          }
        }
      }
      if (kAbl & kAblTrace) t_loop = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
      if (kAbl & kAblDefer) k1_drain<kC>(x, t, ob, S);
      if (kAbl & kAblLoadOnly) {
        t.nl = static_cast<uint32_t>(t.kw1);
        t.kw1 = 0;
      }
      flush_kw(x.kwmask, kw_words, t.f, t.kw0, t.kw1);
      if (x.primary) nl_count[t.ci] = static_cast<uint16_t>(t.nl);   // the range's last chunk
      if (kAbl & kAblTrace) t_kw = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
    }
    // flush this wave's hit buffer (the wave has reconverged here)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t n = min(*x.w_hitcnt, wave_hits);
    uint32_t b0 = 0, o0 = 0;
    if (lane == 0 && n) {
      b0 = atomicAdd(x.b_hitcnt, n);
      if (b0 + n > region_cap) o0 = atomicAdd(x.over_cnt, b0 + n - max(b0, region_cap));
    }
    b0 = __shfl(b0, 0);
    o0 = __shfl(o0, 0);
    const uint32_t spill_from = max(b0, region_cap);
    for (uint32_t i = lane; i < n; i += 64) {
      const uint32_t h = x.w_hits[i];
      const unsigned long long v = ((x.item_base + (h >> kAnchorBits)) << 24) | (h & ((1u << kAnchorBits) - 1));
      if (b0 + i < region_cap) {
        x.hits[b0 + i] = v;
      } else {
        const uint32_t oi = o0 + (b0 + i - spill_from);
        if (oi < x.over_cap) x.over[oi] = v;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if ((kAbl & kAblTrace) && lane == 0 && item < kTraceItemCap) {
      uint32_t* r = trc + 4 * gridDim.x + kTraceItemWords * item;
      r[0] = t_item;
      r[1] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
      r[2] = (kU << 24) | (blockIdx.x << 8) | wid;
      r[3] = t_setup;
      r[4] = t_loop;
      r[5] = t_kw;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) block_hits[blockIdx.x] = s_block[0];
  if ((kAbl & kAblTrace) && threadIdx.x == 0) trc[4 * blockIdx.x + 2] = static_cast<uint32_t>(__builtin_amdgcn_s_memrealtime());
}

// K1 builds: the product's default (4560, K1 and K1c: 464 until round 5,
// plus the fast word step for the words of a boundary line that lie wholly
// in one file -- config-1 files 250 MB launch 0.249 -> 0.229 ms, image-layer
// files 0.277 -> 0.227 ms, config 2 unchanged, profiles/r5d_*).  The measurement
// builds of the DESIGN.md 4.1 ablations (kAbl bits; tools/k1_probe.py
// --variants 3:ABL) exist only in the probe library
// (python -m trivy_amd.build --probe -> libtrivysecret_probe.so, -DTSG_K1_PROBE).
constexpr int kK1Default = 4560;
const void* k1_kernel(int abl, bool compressed) {
  if (compressed) {
    if (abl == kK1Default) return reinterpret_cast<const void*>(&tsg_k1_scan_v3<1024, kK1Default, true>);
#ifdef TSG_K1_PROBE
    if (abl == (kK1Default | kAblCRowOnly)) return reinterpret_cast<const void*>(&tsg_k1_scan_v3<1024, kK1Default | kAblCRowOnly, true>);
    if (abl == (kK1Default | kAblCNoSelect)) return reinterpret_cast<const void*>(&tsg_k1_scan_v3<1024, kK1Default | kAblCNoSelect, true>);
#endif
    return nullptr;
  }
  switch (abl) {
#define TSG_K1_V3(A) case (A): return reinterpret_cast<const void*>(&tsg_k1_scan_v3<1024, (A), false>);
    TSG_K1_V3(kK1Default)
#ifdef TSG_K1_PROBE
    TSG_K1_V3(0) TSG_K1_V3(16) TSG_K1_V3(18) TSG_K1_V3(20) TSG_K1_V3(24) TSG_K1_V3(32) TSG_K1_V3(48)
    TSG_K1_V3(80) TSG_K1_V3(144) TSG_K1_V3(208) TSG_K1_V3(272) TSG_K1_V3(400) TSG_K1_V3(448)
    TSG_K1_V3(464) TSG_K1_V3(465) TSG_K1_V3(466) TSG_K1_V3(468) TSG_K1_V3(472) TSG_K1_V3(496) TSG_K1_V3(976) TSG_K1_V3(1488)
    TSG_K1_V3(2448) TSG_K1_V3(2512) TSG_K1_V3(4592) TSG_K1_V3(8656) TSG_K1_V3(12752)
    TSG_K1_V3(4561) TSG_K1_V3(4562) TSG_K1_V3(5072) TSG_K1_V3(65536 + 4560) TSG_K1_V3(131072 + 4560) TSG_K1_V3(131072 + 4592)
    TSG_K1_V3(262144 + 464) TSG_K1_V3(262144 + 4592) TSG_K1_V3(262144 + 4560)
    TSG_K1_V3(524288 + 4560) TSG_K1_V3(524288 + 262144 + 4560) TSG_K1_V3(524288 + 4592)
    TSG_K1_V3(1048576 + 4560) TSG_K1_V3(1048576 + 262144 + 4560)
    TSG_K1_V3(2097152 + 4560) TSG_K1_V3(4194304 + 4560) TSG_K1_V3(4194304 + 262144 + 4560)
#endif
#undef TSG_K1_V3
    default: return nullptr;
  }
}

// ==== host side: K1's build hash (bench.py k1_build) ends here -- a
// committed traffic measurement applies to that code

template <typename T>
bool dev_upload(const std::vector<T>& v, T** out, std::string* err) {
  size_t n = std::max<size_t>(v.size(), 1) * sizeof(T);
  HIP_OK(hipMalloc(reinterpret_cast<void**>(out), n + 16));
  HIP_OK(hipMemset(*out, 0, n + 16));
  if (!v.empty()) HIP_OK(hipMemcpy(*out, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return true;
}

template <typename T>
bool ensure(T** p, size_t* cap, size_t n, std::string* err) {
  if (*cap >= n && *p) return true;
  if (*p) HIP_OK(hipFree(*p));
  *p = nullptr;
  size_t want = std::max<size_t>(n, 1);
  HIP_OK(hipMalloc(reinterpret_cast<void**>(p), want * sizeof(T) + 64));
  *cap = want;
  return true;
}

// Default K1 chunk for a launch of `bytes` on `lanes` lanes (CUs x 1024).  K1
// walks ranges of 1-4 chunks per lane (guided schedule; 1-8 with top8): its
// chunk is the '\n'-count granularity and the last round's range.  1 KiB
// for launches of 2 GiB and more with top8 (2 KiB without: measured r2r,
// 3.34 vs 3.21 TB/s at 4 GB against 1 KiB with 4-chunk ranges).  Below 2 GiB a
// lane walks ~13 MB/s whatever the load, so a small launch is as fast as its
// lanes' ranges are short and evenly dealt (round 5: a 250 MB launch 0.249 ->
// 0.231 ms with 512-B chunks against 1 KiB, 1 GB 0.583 -> 0.529 ms).  Round 6
// (profiles/r8h_*, config-1 files): the chunk that fits the launch in exactly
// one round of one-chunk ranges when one of <= 512 B does (100 MB: 384 B,
// 0.079 ms, against 0.096 with 256 B; 125 MB: 512 B, 0.097 against 0.111 with
// the rounded-down 384 B, whose 1.24 chunks per lane left a second round of
// 2-chunk ranges); 256 B up to 512 MB (150 MB 0.126 -> 0.104 ms against 512 B,
// 200 MB 0.135 -> 0.121, 300 MB 0.176 -> 0.162, 400 MB equal, 500 MB 0.253 ->
// 0.235); 512 B above (600 MB equal, 800 MB 0.331 against 0.341 with 256 B,
// 1.5 GB 0.551 against 0.58).
// Resident pieces keep 512 B there: a piece's per-chunk '\n' counts are read
// back and summed by the confirmation after its K2, on the step's critical
// path for the last piece, and 256-B chunks double them (1 GB of config-1
// files in three resident pieces: 1.45-1.46 ms per step at 512 B, 1.58 at
// 256, profiles/r9h_*).
uint32_t k1_chunk_for(uint64_t bytes, uint32_t lanes, int top8, bool resident) {
  if (bytes >= (2ull << 30)) return top8 ? 1024 : 2048;   // (top8 != 0)
  const uint64_t l = std::max<uint32_t>(lanes, 1);
  const uint64_t one_round = ((bytes + l - 1) / l + 127) & ~uint64_t(127);   // chunks <= lanes
  if (one_round <= 512) return static_cast<uint32_t>(std::max<uint64_t>(128, one_round));
  return bytes <= (512ull << 20) && !resident ? 256 : 512;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

// Device tables of one scan DFA group (one K1 launch per group).
struct K1Group {
  uint16_t* next = nullptr;    // pre-multiplied uint16 row offsets, row stride `stride`
  uint8_t* cls = nullptr;      // byte -> class * 2
  OutMeta* meta = nullptr;
  uint32_t* list = nullptr;
  uint32_t nmeta = 0, nlist = 0, table_words16 = 0, stride = 0, ostride = 0, nclasses = 0, first_out = 0;
  uint32_t kw_base = 0, warm_lines = 0, warm_lines64 = 0;
  size_t meta_bytes = 0;
  bool in_lds = false;
  bool compressed = false;     // K1c table (prefilter.h CompressedScan): first_out holds the start state's value
};

// The compiled rule tables on one device plus that device's pool of lanes.
struct DeviceTables {
  int device = 0;
  int sms = 256;
  std::vector<K1Group> k1g;
  K2Anchor* anchors = nullptr;                 // K2's per-anchor records
  uint32_t* rule_kw = nullptr;
  uint16_t* v_next = nullptr;
  uint8_t* v_cls = nullptr;
  uint32_t kw_words = 1;
  std::mutex mu;                               // guards the lane pool and lds_set
  std::vector<std::pair<const void*, int>> lds_set;   // K1 builds whose dynamic-LDS limit is set (per device)
  std::vector<std::unique_ptr<Lane>> lanes;
  std::vector<Lane*> free_lanes;
  ~DeviceTables();
};

// One in-flight call's resources on one device: its own streams (compute +
// copy), timing events, the two-slot upload ring and every per-batch scratch
// buffer, so concurrent calls never share mutable GPU state.
struct PinnedBuf {
  void* p = nullptr;     // host address
  void* d = nullptr;     // the same memory as the device sees it
  size_t cap = 0;
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

// host-mapped, coherent (fine-grained) pinned memory for tsg_readback
bool ensure_pinned(PinnedBuf* b, size_t bytes, std::string* err) {
  if (b->p && b->cap >= bytes) return true;
  if (b->p) HIP_OK(hipHostFree(b->p));
  b->p = b->d = nullptr;
  b->cap = 0;
  const size_t want = (std::max<size_t>(bytes + bytes / 4, 256) + 63) & ~size_t(63);
  HIP_OK(hipHostMalloc(&b->p, want + 64, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_OK(hipHostGetDevicePointer(&b->d, b->p, 0));
  b->cap = want;
  return true;
}

// Readbacks of one segment: dwords of device buffers into host-mapped
// pinned buffers, queued together as one tsg_readback launch on stream s
struct Readbacks {
  RbList L{};
  int n = 0;
  size_t max_words = 0;
  void add(const void* src, const PinnedBuf& b, size_t nwords, const uint32_t* d_count = nullptr, uint32_t per_count = 0) {
    if (nwords == 0) return;
    L.r[n++] = RbRegion{static_cast<const uint4*>(src), static_cast<uint4*>(b.d), d_count,
                        static_cast<uint32_t>(nwords), per_count};
    max_words = std::max(max_words, nwords);
  }
  bool launch(hipStream_t s, std::string* err) {
    if (n == 0) return true;
    const uint32_t blocks = static_cast<uint32_t>(std::min<size_t>(1024, (max_words / 4 + 256) / 256));
    hipLaunchKernelGGL(tsg_readback, dim3(blocks, n), dim3(256), 0, s, L);
    HIP_OK(hipGetLastError());
    return true;
  }
};

// dwords of src (device) into b (host-mapped) on stream s
bool readback(const void* src, const PinnedBuf& b, size_t nwords, const uint32_t* d_count, uint32_t per_count,
              hipStream_t s, std::string* err) {
  Readbacks rb;
  rb.add(src, b, nwords, d_count, per_count);
  return rb.launch(s, err);
}

// Two drivers of one device (resident batches): each queues its segment's
// K1 + K2 behind the other's last K2 (the event below), so the device runs
// the segments' passes back to back -- a K1 takes every CU's LDS, a K2
// launched beside it would wait for it -- while the other driver's readback,
// copy-out and launch overhead overlap them instead of leaving the device
// idle between segments (0.17-0.21 ms per piece, profiles/rd5c_bench_c2prof.log).
// Drivers in this mode poll their event between short sleeps (no spinning
// core taken from the confirm pool).
struct K1Chain {
  std::mutex mu;
  hipEvent_t last = nullptr;                    // end of the last K2 queued on the device
};

// A small batch in pinned host memory staged by the segment prologue kernel
// (tsg_prologue) instead of the copy engine: device views of its bytes and
// offsets, and their destinations.
struct StageIn {
  const uint8_t* src = nullptr; uint8_t* dst = nullptr; uint64_t bytes = 0;
  const uint8_t* off_src = nullptr; uint8_t* off_dst = nullptr; uint64_t off_bytes = 0;
};
constexpr uint64_t kDirectStageBytes = 1u << 20;     // batches up to this size (and pinned) are staged by the prologue

struct Lane {
  int device = 0;
  hipStream_t compute = nullptr, copy = nullptr;
  hipEvent_t ev[4] = {};                        // K1 start/end, K2 start/end (compute stream)
  hipEvent_t ev_sync = nullptr;                 // blocking-sync event (K1Chain drivers)
  const std::atomic<bool>* pool_idle = nullptr; // set by a scan's driver: its confirm pool has no work
  hipEvent_t up_begin[2] = {}, up_done[2] = {}; // upload ring slot: H2D start / done (copy stream)
  hipEvent_t anchor = nullptr;                   // TSG_HOST_PROFILE: start of a scan() on the copy stream
  uint8_t* ring[2] = {nullptr, nullptr};
  size_t ring_cap[2] = {0, 0};
  uint64_t* d_off = nullptr; size_t d_off_cap = 0;
  // uploaded data: the segment's offsets travel on the copy stream with its
  // bytes, from pinned staging (a pageable copy of >~64 KB on the compute
  // stream is staged through the copy engine and queues behind the next
  // segment's upload: measured, config 1's first K1 waited 8.8 ms)
  uint64_t* off_slot[2] = {nullptr, nullptr}; size_t off_slot_cap[2] = {0, 0};
  uint64_t* h_off_pin[2] = {nullptr, nullptr}; size_t h_off_pin_cap[2] = {0, 0};
  // readbacks land in pinned memory (a pageable D2H is staged through a copy
  // engine and at times waited behind the next segment's upload: r3q/r3u
  // config 2, up to 22 ms between K2 done and the results on the host)
  PinnedBuf rb_bh, rb_c2, rb_cands, rb_ff, rb_nl;
  uint32_t* d_kw = nullptr; size_t d_kw_cap = 0;
  unsigned long long* d_hits = nullptr; size_t d_hits_cap = 0;
  unsigned long long* d_over = nullptr; size_t d_over_cap = 0;   // hits past a full region (any workgroup)
  uint32_t* d_bh = nullptr; size_t d_bh_cap = 0;    // hits written per K1 workgroup (its region of d_hits)
  CandDev* d_cands = nullptr; size_t d_cands_cap = 0;
  uint16_t* d_nl = nullptr; size_t d_nl_cap = 0;   // '\n' per K1 chunk (chunk <= 32 KiB)
  uint32_t* d_cf = nullptr; size_t d_cf_cap = 0;   // per K1 chunk: a file at or before its first byte (K2's file lookup)
  uint32_t* d_ff = nullptr; size_t d_ff_cap = 0;
  uint32_t* d_ob = nullptr; size_t d_ob_cap = 0;    // K1 v3 deferred-output slots (kOutSlots per thread)
  uint32_t* d_fidx = nullptr; size_t d_fidx_cap = 0;   // K1's file index (tsg_file_index): one entry per 64 KiB
  unsigned long long* d_k2s = nullptr;              // TSG_K2_STATS: per-rule K2 counters (4 per rule)
  unsigned int* d_cnt = nullptr;
  uint8_t* d_cr = nullptr; size_t d_cr_cap = 0;     // CR strip scratch (crstrip.hip)
  size_t hit_cap = 1 << 20, cand_cap = 1 << 18, over_cap = 1 << 18;
  double k2_maxr_per_byte = 0;                       // K2 grid of the next segment: the last one's fullest region
  uint64_t k2_over_est = 0;                          // per byte, and its overflow hit count
  ~Lane();
};

// GPU results of one segment, handed from a device driver thread to the
// host confirmer.
struct GpuOut {
  std::vector<CandDev> cands;   // (file, rule, start) candidates, unsorted
  std::vector<uint16_t> nl;     // '\n' count per K1 chunk
  std::vector<uint32_t> ff;     // per-file flags (fold-special content)
  uint32_t chunk = 0;           // K1 chunk bytes of this segment (nl[] granularity)
  // deferred copy-out (run_segment with defer_copy): the three arrays are
  // still in the lane's pinned readback buffers; finish_copy() moves them
  // here before the lane's next readback is queued
  const CandDev* rb_cands = nullptr;
  const uint32_t* rb_ff = nullptr;
  const uint16_t* rb_nl = nullptr;
  size_t n_cands = 0, n_ff = 0, n_nl = 0;
  bool deferred = false;
  void finish_copy() {
    if (!deferred) return;
    cands.assign(rb_cands, rb_cands + n_cands);
    ff.assign(rb_ff, rb_ff + n_ff);
    nl.assign(rb_nl, rb_nl + n_nl);
    deferred = false;
  }
  // the confirmation's plan (plan_confirm): candidates grouped per file, the
  // files to confirm (largest first) and the rest.  (Built on the driver
  // thread it delayed the next piece's launch by as much as it saved the
  // confirming thread: profiles/rd4q_bench_c3prof.log; it is now built while
  // the next piece's passes run.)
  bool planned = false;
  std::vector<uint32_t> per_file, work, light;
  std::vector<CandDev> sorted;
};

// One call's host confirm resources.
// The pool is created at the call's first confirmation that needs it: per-file
// Scan batches (a few files, confirmed inline on the calling thread) never
// start one, so the queue's up to max_inflight concurrent batches hold a lane
// each but no idle confirm threads.
struct CallCtx {
  std::unique_ptr<ThreadPool> pool;
  int nt = 1;
  ThreadPool& get() {
    if (!pool || pool->size() != nt) pool.reset(new ThreadPool(nt));
    return *pool;
  }
};

// A self-contained sub-batch: files [f0, f0 + in.nfiles) of the call's
// batch, offsets rebased to 0, data pointers advanced to its first byte.
struct Engine::Segment {
  BatchInput in;
  std::vector<uint64_t> off;
  uint32_t f0 = 0;
  uint64_t b0 = 0, bytes = 0;
  // resident pieces: file 0 of `in` is a lead of the bytes between the
  // 256-byte boundary below the piece's first file and that file (the tail of
  // the previous piece), so K1's lines are aligned as on the pinned path; its
  // results are dropped.  lead_* hold the shifted path / length / binary arrays.
  uint32_t lead = 0;
  std::vector<const char*> lead_paths;
  std::vector<uint32_t> lead_lens;
  std::vector<uint8_t> lead_bin;
};

DeviceTables::~DeviceTables() {
  hipSetDevice(device);
  lanes.clear();
  void* ps[] = {anchors, rule_kw, v_next, v_cls};
  for (void* p : ps) if (p) hipFree(p);
  for (K1Group& g : k1g) {
    void* gs[] = {g.next, g.cls, g.meta, g.list};
    for (void* p : gs) if (p) hipFree(p);
  }
}

Lane::~Lane() {
  hipSetDevice(device);
  if (compute) hipStreamSynchronize(compute);
  if (copy) hipStreamSynchronize(copy);
  for (uint64_t* h : h_off_pin) if (h) hipHostFree(h);
  for (PinnedBuf* b : {&rb_bh, &rb_c2, &rb_cands, &rb_ff, &rb_nl}) if (b->p) hipHostFree(b->p);
  void* ps[] = {ring[0], ring[1], off_slot[0], off_slot[1], d_off, d_kw, d_hits, d_over, d_bh, d_cands, d_nl, d_cf, d_ff, d_ob, d_cnt, d_k2s, d_cr, d_fidx};
  for (void* p : ps) if (p) hipFree(p);
  for (auto& e : ev) if (e) hipEventDestroy(e);
  if (ev_sync) hipEventDestroy(ev_sync);
  if (anchor) hipEventDestroy(anchor);
  for (int i = 0; i < 2; ++i) {
    if (up_begin[i]) hipEventDestroy(up_begin[i]);
    if (up_done[i]) hipEventDestroy(up_done[i]);
  }
  if (compute) hipStreamDestroy(compute);
  if (copy) hipStreamDestroy(copy);
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

bool readback_probe(uint32_t nwords, uint32_t count, uint32_t per_count, uint32_t* copied, std::string* err) {
  if (device_count() <= 0) { *err = "no HIP device available"; return false; }
  if (nwords == 0 || nwords > (64u << 20)) { *err = "nwords out of range"; return false; }
  HIP_OK(hipSetDevice(0));
  const size_t n4 = (static_cast<size_t>(nwords) + 3) & ~size_t(3);   // the kernel moves 16-byte granules
  std::vector<uint32_t> h(n4 + 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint32_t>(i + 1);
  uint32_t* d_src = nullptr;
  uint32_t* d_cnt = nullptr;
  PinnedBuf dst;
  bool ok = false;
  std::string e2;
  do {
    if (hipMalloc(&d_src, h.size() * 4) != hipSuccess || hipMalloc(&d_cnt, 4) != hipSuccess) { e2 = "hipMalloc"; break; }
    if (hipMemcpy(d_src, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_cnt, &count, 4, hipMemcpyHostToDevice) != hipSuccess) { e2 = "hipMemcpy"; break; }
    if (!ensure_pinned(&dst, h.size() * 4, &e2)) break;
    std::memset(dst.p, 0, dst.cap);
    if (!readback(d_src, dst, nwords, d_cnt, per_count, nullptr, &e2)) break;
    if (hipDeviceSynchronize() != hipSuccess) { e2 = "hipDeviceSynchronize"; break; }
    const uint32_t* got = dst.as<const uint32_t>();
    uint32_t n = 0;
    while (n < n4 && got[n] == n + 1) ++n;
    *copied = n;
    ok = true;
  } while (false);
  if (d_src) hipFree(d_src);
  if (d_cnt) hipFree(d_cnt);
  if (dst.p) hipHostFree(dst.p);
  if (!ok) *err = e2;
  return ok;
}

namespace {

// Upload the prefilter's tables to one device.
bool build_tables(const Prefilter& pf, DeviceTables* dt, std::string* err) {
  HIP_OK(hipSetDevice(dt->device));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dt->device) == hipSuccess) dt->sms = prop.multiProcessorCount;
  if (pf.anchors.size() >= (1u << kAnchorBits)) { *err = "too many anchor literals for K1's hit encoding"; return false; }
  dt->kw_words = std::max<uint32_t>(1, (pf.nkw + 31) / 32);
  if (pf.compressed.ok) {
    // K1c: every pattern in one compressed table, one pass (replaces the groups)
    const CompressedScan& c = pf.compressed;
    K1Group g;
    g.compressed = true;
    g.nclasses = c.nclasses;
    g.stride = c.row_stride;
    g.first_out = c.state_val[0];
    g.kw_base = 0;
    const uint32_t warm = c.max_pattern_bytes > 0 ? c.max_pattern_bytes - 1 : 0;
    g.warm_lines = (warm + 127) / 128;
    g.warm_lines64 = (warm + 63) / 64;
    std::vector<uint32_t> img = c.image;
    img.resize((img.size() + 3) & ~size_t(3), 0);
    g.table_words16 = static_cast<uint32_t>(img.size() * 2);
    g.nmeta = static_cast<uint32_t>(c.outs.size());
    g.nlist = static_cast<uint32_t>(c.out_list.size());
    g.meta_bytes = 0;                                        // outputs stay in global memory
    g.in_lds = kK1HitLdsMin + 256 + img.size() * 4 <= kLdsBytes;
    std::vector<OutMeta> meta;
    for (const auto& o : c.outs) meta.push_back(OutMeta{o.kw0, o.kw1, o.list_begin, o.list_count});
    std::vector<uint8_t> cls(c.cls4, c.cls4 + 256);
    if (!dev_upload(img, reinterpret_cast<uint32_t**>(&g.next), err) || !dev_upload(cls, &g.cls, err) ||
        !dev_upload(meta, &g.meta, err) || !dev_upload(c.out_list, &g.list, err)) {
      return false;
    }
    dt->kw_words = std::max<uint32_t>(dt->kw_words, 4);
    dt->k1g.push_back(g);
  }
  for (const ScanDfa& sd : pf.groups) {
    if (pf.compressed.ok) break;
    K1Group g;
    // scan table with an odd dword row stride: next[s*stride + c] then spreads
    // the same class of different states over different LDS banks (a 64-class
    // row is 32 dwords, which would put every state's class c in one bank).
    // Silent rows first (stride S), then output rows (stride So): slot C of an
    // output row holds the output-state index (kept for the layout), slots
    // S..S+9 its metadata inline (v3: keyword masks and list in the same LDS
    // round trip as the row address)
    const uint32_t C = sd.t.nclasses;
    const uint32_t stride = k1_row_stride(C);
    const uint32_t ostride = k1_out_row_stride(C);
    const uint32_t fo = sd.first_out_state;
    g.stride = stride;
    g.nclasses = C;
    g.first_out = fo * stride / 2;               // row offsets in dwords (stride is even)
    g.kw_base = sd.kw_base;
    const uint32_t warm = sd.max_pattern_bytes > 0 ? sd.max_pattern_bytes - 1 : 0;
    g.warm_lines = (warm + 127) / 128;          // warm-up = whole 128-byte lines before the chunk (128-B line builds)
    g.warm_lines64 = (warm + 63) / 64;          // v3 (64-byte lines): whole 64-byte lines
    // entries hold the next state's row offset: the DFA chain is then one
    // add + one LDS read per byte (no multiply)
    if (k1_table_words16(sd) > 2 * 65535) {
      *err = "scan DFA group too large for 16-bit pre-multiplied dword offsets";
      return false;
    }
    if (C > 127) { *err = "scan DFA has more than 127 byte classes"; return false; }
    auto row = [&](uint32_t st) { return st < fo ? st * stride : fo * stride + (st - fo) * ostride; };
    std::vector<uint16_t> sn(k1_table_words16(sd), 0);
    for (uint32_t st = 0; st < sd.t.nstates; ++st) {
      for (uint32_t c = 0; c < C; ++c)
        sn[row(st) + c] = static_cast<uint16_t>(row(sd.t.next[static_cast<size_t>(st) * C + c]) / 2);
      if (st >= fo) sn[row(st) + C] = static_cast<uint16_t>(st - fo);
    }
    // per output state: keyword masks (ids kw_base .. kw_base+127) + list of other output ids
    std::vector<OutMeta> meta;
    std::vector<uint32_t> olist;
    for (uint32_t o = 0; o + 1 < sd.out_off.size(); ++o) {
      OutMeta om{0, 0, static_cast<uint32_t>(olist.size()), 0};
      for (uint32_t k = sd.out_off[o]; k < sd.out_off[o + 1]; ++k) {
        const uint32_t id = sd.out_ids[k];
        if (id < pf.nkw && id >= g.kw_base && id < g.kw_base + 64) om.kw0 |= 1ull << (id - g.kw_base);
        else if (id < pf.nkw && id >= g.kw_base + 64 && id < g.kw_base + 128) om.kw1 |= 1ull << (id - g.kw_base - 64);
        else olist.push_back(id);
      }
      om.list_count = static_cast<uint32_t>(olist.size()) - om.list_begin;
      if (om.list_begin > 0xffff || om.list_count > 0xffff) { *err = "scan DFA output list too long"; return false; }
      meta.push_back(om);
      uint16_t* m = &sn[row(fo + o) + stride];
      for (int k = 0; k < 4; ++k) {
        m[k] = static_cast<uint16_t>(om.kw0 >> (16 * k));
        m[4 + k] = static_cast<uint16_t>(om.kw1 >> (16 * k));
      }
      m[8] = static_cast<uint16_t>(om.list_begin);
      m[9] = static_cast<uint16_t>(om.list_count);
    }
    g.ostride = ostride;
    g.nmeta = static_cast<uint32_t>(meta.size());
    g.nlist = static_cast<uint32_t>(olist.size());
    g.meta_bytes = (olist.size() * 4 + 15) & ~size_t(15);   // in LDS: the output list (metadata is inline)
    g.table_words16 = static_cast<uint32_t>(sn.size());
    // LDS: per-wave hit buffers (16 waves) + counters + scan table + class map + output metadata
    g.in_lds = kK1HitLdsMin + ((static_cast<size_t>(g.table_words16) * 2 + 15) & ~size_t(15)) + 256 + g.meta_bytes <= kLdsBytes;
    sn.resize(((sn.size() * 2 + 15) / 16) * 8, 0);
    // K1's class map holds class * 2 (see k1_step)
    std::vector<uint8_t> cls(256);
    for (int b = 0; b < 256; ++b) cls[b] = static_cast<uint8_t>(sd.t.byte_class[b] * 2);
    if (!dev_upload(sn, &g.next, err) || !dev_upload(cls, &g.cls, err) || !dev_upload(meta, &g.meta, err) ||
        !dev_upload(olist, &g.list, err)) {
      return false;
    }
    dt->kw_words = std::max<uint32_t>(dt->kw_words, g.kw_base / 32 + 4);   // a group's masks span 4 words from kw_base
    dt->k1g.push_back(g);
  }
  // K2: the verify DFAs' transitions with the accept flag in bit 15, and
  // one record per anchor (its rule's fields and DFA offsets inline)
  std::vector<uint16_t> vn;
  std::vector<uint8_t> vc;
  std::vector<uint32_t> v_next_off, v_cls_off;
  for (const auto& t : pf.verify) {
    if (t.nstates > kVState || t.nclasses > 0xffff || t.dead > 0xffff) { *err = "verify DFA too large for K2's records"; return false; }
    v_next_off.push_back(static_cast<uint32_t>(vn.size()));
    v_cls_off.push_back(static_cast<uint32_t>(vc.size()));
    for (uint16_t x : t.next) vn.push_back(static_cast<uint16_t>(x | (t.accept[x] ? kVAcc : 0u)));
    vc.insert(vc.end(), t.byte_class, t.byte_class + 256);
  }
  std::vector<K2Anchor> an;
  for (const auto& a : pf.anchors) {
    const RuleGpuInfo& r = pf.rules[a.rule];
    K2Anchor k{};
    k.rule = a.rule; k.min_len = a.min_len; k.max_len = a.max_len; k.dmin = a.dmin; k.dmax = a.dmax;
    k.kw_begin = r.kw_begin; k.kw_count = r.kw_count;
    k.kw0 = r.kw_count ? pf.rule_kw[r.kw_begin] : 0;
    k.verify_limit = r.verify_limit;
    uint32_t flags = r.mode | (r.gate_on_gpu ? 0x100u : 0u) | (r.always_gate ? 0x200u : 0u);
    if (r.mode == 0 || r.mode == 4) {
      const DfaTable& v = pf.verify[r.verify_dfa];
      k.v_next = v_next_off[r.verify_dfa]; k.v_cls = v_cls_off[r.verify_dfa];
      k.v_ncls_dead = v.nclasses | (v.dead << 16);
      if (!v.accept.empty() && v.accept[0]) flags |= 0x400u;
    }
    if (r.mode == 4) {
      const DfaTable& v = pf.verify[r.rev_dfa];
      k.r_next = v_next_off[r.rev_dfa]; k.r_cls = v_cls_off[r.rev_dfa];
      k.r_ncls_dead = v.nclasses | (v.dead << 16);
    }
    k.flags = flags;
    an.push_back(k);
  }
  return dev_upload(an, &dt->anchors, err) && dev_upload(pf.rule_kw, &dt->rule_kw, err) &&
         dev_upload(vn, &dt->v_next, err) && dev_upload(vc, &dt->v_cls, err);
}

// Device of a device pointer (-1: not a device allocation).
int device_of(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) { (void)hipGetLastError(); return -1; }
  if (a.type != hipMemoryTypeDevice) return -1;
  return a.device;
}

void add_stats(ScanStats* a, const ScanStats& s) {
  a->k1_ms += s.k1_ms; a->k2_ms += s.k2_ms; a->h2d_ms += s.h2d_ms; a->d2h_ms += s.d2h_ms;
  a->hits += s.hits; a->candidates += s.candidates; a->k1_launches += s.k1_launches;
  a->k1_blocks = s.k1_blocks; a->k1_threads = s.k1_threads; a->chunk_bytes = s.chunk_bytes;
  a->table_in_lds = s.table_in_lds;
}

}  // namespace

std::unique_ptr<Engine> Engine::create(std::shared_ptr<const Ruleset> rs, const std::vector<int>& devices,
                                       std::string* err) {
  const int n = device_count();
  if (n <= 0) { *err = "no HIP device available (the GPU engine has no CPU fallback)"; return nullptr; }
  if (devices.empty()) { *err = "no device selected"; return nullptr; }
  for (int d : devices) {
    if (d < 0 || d >= n) { *err = "HIP device index out of range"; return nullptr; }
  }
  std::unique_ptr<Engine> e(new Engine());
  e->rs_ = std::move(rs);
  e->devices_ = devices;
  if (!build_prefilter(*e->rs_, &e->pf_, err)) return nullptr;
  if (const char* c = std::getenv("TSG_PIECES")) {
    const long v = std::atol(c);
    if (v >= 1 && v <= 64) e->pieces_ = static_cast<uint32_t>(v);
  }
  if (const char* c = std::getenv("TSG_FIRST_PIECE")) {
    const double v = std::atof(c);
    if (v > 0.0 && v < 1.0) e->first_piece_ = v;
  }
  if (const char* c = std::getenv("TSG_FIRST_PIECE_FEW")) {
    const double v = std::atof(c);
    if (v > 0.0 && v < 1.0) e->first_piece_few_ = v;
  }
  if (const char* c = std::getenv("TSG_LAST_PIECE")) {
    const double v = std::atof(c);
    if (v >= 0.0 && v < 0.5) e->last_piece_ = v;
  }
  if (const char* c = std::getenv("TSG_MIN_PIECE_BYTES")) {
    const long long v = std::atoll(c);
    if (v >= 1) e->min_piece_ = static_cast<uint64_t>(v);
  }
  if (const char* c = std::getenv("TSG_SEGMENT_BYTES")) {
    const long long v = std::atoll(c);
    if (v >= 4096) e->segment_ = static_cast<uint64_t>(v);
  }
  if (const char* c = std::getenv("TSG_SEGMENT_MIN")) {
    const long long v = std::atoll(c);
    if (v >= 4096) e->segment_min_ = static_cast<uint64_t>(v);
  }
  if (const char* c = std::getenv("TSG_SEGMENT_BALANCED")) e->balanced_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("TSG_SEGMENT_TAIL")) {
    const long long v = std::atoll(c);
    if (v >= 0) e->segment_tail_ = static_cast<uint64_t>(v);
  }
  if (const char* c = std::getenv("TSG_K1_ABL")) e->k1_abl_ = std::atoi(c);   // K1 measurement builds (kAbl bits)
  if (const char* c = std::getenv("TSG_K2_STATS")) e->k2_stats_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("TSG_K2_ABL")) e->k2_abl_ = std::atoi(c) & (kK2Trace | kK2NoWalk);   // probe library builds
  if (const char* c = std::getenv("TSG_RESIDENT_DRIVERS")) e->resident_drivers_ = std::max(1, std::atoi(c));
  if (const char* c = std::getenv("TSG_CHAIN_K1")) e->chain_k1_ = std::max(0, std::min(2, std::atoi(c)));
  if (const char* c = std::getenv("TSG_READBACK_DMA")) e->readback_dma_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("TSG_K1_FILE_INDEX")) e->file_index_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("TSG_K1_RESERVE_CUS")) e->k1_reserve_cus_ = static_cast<uint32_t>(std::max(0, std::min(64, std::atoi(c))));
  if (const char* c = std::getenv("TSG_CONFIRM_PREFETCH")) e->confirm_prefetch_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("TSG_POLL_YIELD")) e->poll_yield_ = std::atoi(c) != 0;
  if (const char* c = std::getenv("TSG_POP_SPIN_US")) e->pop_spin_us_ = std::max(0, std::min(std::atoi(c), 100000));
  if (const char* c = std::getenv("TSG_HOST_PROFILE")) e->host_profile_ = std::atoi(c) != 0;
  if (e->host_profile_) g_scan_prof_on.store(true, std::memory_order_relaxed);
  if (const char* c = std::getenv("TSG_K1_TAIL_ROUNDS")) {
    const int v = std::atoi(c);
    if (v >= 0 && v <= 16) e->k1_tail_rounds_ = static_cast<uint32_t>(v);
  }
  if (const char* c = std::getenv("TSG_K1_TOP8")) e->k1_top8_ = std::max(0, std::min(2, std::atoi(c)));
  if (const char* c = std::getenv("TSG_K2_HITS_PER_THREAD")) {
    const int v = std::atoi(c);
    if (v >= 1 && v <= 64) e->k2_hits_per_thread_ = static_cast<uint32_t>(v);
  }
  if (const char* c = std::getenv("TSG_K1_CHUNK")) {
    // K1's LDS hit record keeps (offset in the wave item) << kAnchorBits in
    // 32 bits and a wave item spans 64 lanes x 4 chunks: larger chunks are
    // clamped so the offset cannot wrap
    const long v = std::atol(c);
    if (v >= 128 && v % 128 == 0) e->chunk_ = static_cast<uint32_t>(std::min<long>(v, k1_max_chunk(kItemChunks)));
  }
  for (int d : devices) {
    std::unique_ptr<DeviceTables> dt(new DeviceTables());
    dt->device = d;
    if (!build_tables(e->pf_, dt.get(), err)) return nullptr;
    e->dev_.push_back(std::move(dt));
  }
  return e;
}

Engine::~Engine() {
  if (k2_stats_ && !k2s_.empty()) {
    // TSG_K2_STATS: per-rule K2 work of every scan of this engine, busiest first
    std::vector<size_t> order(k2s_.size() / kK2Stat);
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t a, size_t b) { return k2s_[kK2Stat * a + 3] > k2s_[kK2Stat * b + 3]; });
    std::string js = "{\"k2_stats\": [";
    bool first = true;
    for (size_t i : order) {
      if (k2s_[kK2Stat * i] == 0) continue;
      const std::string id = i < rs_->rules.size() ? rs_->rules[i].id : "exclude-" + std::to_string(i - rs_->rules.size());
      js += std::string(first ? "" : ", ") + "{\"rule\": \"" + id + "\", \"hits\": " + std::to_string(k2s_[kK2Stat * i]) +
            ", \"gated\": " + std::to_string(k2s_[kK2Stat * i + 1]) + ", \"starts\": " + std::to_string(k2s_[kK2Stat * i + 2]) +
            ", \"bytes\": " + std::to_string(k2s_[kK2Stat * i + 3]) + ", \"max_hit_bytes\": " +
            std::to_string(k2s_[kK2Stat * i + 4]) + "}";
      first = false;
    }
    js += "]}";
    std::fprintf(stderr, "%s\n", js.c_str());
  }
  dev_.clear();
  calls_.clear();
}

Lane* Engine::acquire_lane(DeviceTables& dt, std::string* err) {
  {
    std::lock_guard<std::mutex> lk(dt.mu);
    if (!dt.free_lanes.empty()) {
      Lane* l = dt.free_lanes.back();
      dt.free_lanes.pop_back();
      return l;
    }
  }
  std::unique_ptr<Lane> l(new Lane());
  l->device = dt.device;
  if (hipSetDevice(dt.device) != hipSuccess || hipStreamCreateWithFlags(&l->compute, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&l->copy, hipStreamNonBlocking) != hipSuccess || hipMalloc(&l->d_cnt, kCntBytes) != hipSuccess) {
    *err = "lane setup (streams, counters) failed";
    return nullptr;
  }
  for (auto& ev : l->ev) if (hipEventCreate(&ev) != hipSuccess) { *err = "hipEventCreate failed"; return nullptr; }
  if (k2_stats_) {
    const size_t n = kK2Stat * std::max<size_t>(pf_.rules.size(), 1) * sizeof(unsigned long long);
    if (hipMalloc(&l->d_k2s, n) != hipSuccess || hipMemset(l->d_k2s, 0, n) != hipSuccess) {
      *err = "K2 stats buffer";
      return nullptr;
    }
  }
  if (hipEventCreate(&l->anchor) != hipSuccess) { *err = "hipEventCreate failed"; return nullptr; }
  for (int i = 0; i < 2; ++i) {
    if (hipEventCreate(&l->up_begin[i]) != hipSuccess || hipEventCreate(&l->up_done[i]) != hipSuccess) {
      *err = "hipEventCreate failed";
      return nullptr;
    }
  }
  std::lock_guard<std::mutex> lk(dt.mu);
  dt.lanes.push_back(std::move(l));
  return dt.lanes.back().get();
}

void Engine::release_lane(DeviceTables& dt, Lane* ln) {
  std::lock_guard<std::mutex> lk(dt.mu);
  dt.free_lanes.push_back(ln);
}

CallCtx* Engine::acquire_call() {
  std::lock_guard<std::mutex> lk(call_mu_);
  const int nt = threads_ > 0 ? threads_ : static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
  CallCtx* cc = nullptr;
  if (!free_calls_.empty()) {
    cc = free_calls_.back();
    free_calls_.pop_back();
  } else {
    calls_.emplace_back(new CallCtx());
    cc = calls_.back().get();
  }
  cc->nt = nt;                                   // (the pool itself starts on first use: CallCtx::get)
  return cc;
}

void Engine::footprint(uint32_t* lanes, uint32_t* calls, uint32_t* pool_threads) {
  *lanes = 0;
  for (auto& d : dev_) {
    std::lock_guard<std::mutex> lk(d->mu);
    *lanes += static_cast<uint32_t>(d->lanes.size());
  }
  std::lock_guard<std::mutex> lk(call_mu_);
  *calls = static_cast<uint32_t>(calls_.size());
  *pool_threads = 0;
  for (auto& c : calls_) if (c->pool) *pool_threads += static_cast<uint32_t>(c->pool->size());
}

void Engine::release_call(CallCtx* cc) {
  std::lock_guard<std::mutex> lk(call_mu_);
  free_calls_.push_back(cc);
}

// K1 + K2 + candidate D2H of one segment whose bytes are at d_data on the
// lane's device (resident, or landed by the lane's upload), on the lane's
// compute stream.  Returns when the segment's results are on the host.
bool Engine::run_segment(DeviceTables& dt, Lane& ln, const Segment& sg, const void* d_data_v, const uint64_t* d_off_up,
                         ScanStats* st, GpuOut* out, std::string* err, const std::function<void()>* while_gpu,
                         K1Chain* chain, bool defer_copy, const StageIn* stage_in) {
  const BatchInput& in = sg.in;
  // this call's prologue copies (a small pinned batch, staged offsets): a
  // local, so nothing staged for one call can outlive it on the pooled lane
  // (a stage left on the lane by an early return was copied by the
  // next caller's prologue from a freed pinned buffer)
  StageIn stage = stage_in ? *stage_in : StageIn();
  HIP_OK(hipSetDevice(dt.device));
  const uint64_t total = in.offsets[in.nfiles];
  const uint8_t* d_data = static_cast<const uint8_t*>(d_data_v);
  if ((reinterpret_cast<uintptr_t>(d_data) & 15) != 0) { *err = "device data must be 16-byte aligned"; return false; }
  // top8 for uploaded segments only: HBM-resident pieces, whose K1 runs beside
  // the previous piece's K2 (K1Chain), ran slower with it (config 2 resident
  // 5.55 vs 6.06-6.65 ms per step, K1 3.72 vs 3.80 ms, profiles/r8l_*)
  const int top8_req = sg.in.d_data ? 0 : k1_top8_;
  const uint32_t kChunk = chunk_ ? chunk_ : k1_chunk_for(total, static_cast<uint32_t>(std::max(dt.sms, 1)) * 1024u, top8_req,
                                                         sg.in.d_data != nullptr);
  if (kChunk > k1_max_chunk(kItemChunks) || kChunk % 128 != 0) { *err = "K1 chunk exceeds the hit record's offset range"; return false; }
  // the kU = 8 bulk level (TSG_K1_TOP8) for launches of >= 2 GiB (2: any
  // launch, for tests), while an 8-chunk wave item fits the hit record's
  // offset bits
  const bool top8 = (top8_req == 2 || (top8_req == 1 && total >= (2ull << 30))) && kChunk <= k1_max_chunk(8);
  if ((k1_abl_ & kAblNoLoad) && total < (1u << 20) + 64) { *err = "TSG_K1_ABL no-load build needs a batch of >= 1 MiB"; return false; }
  st->chunk_bytes = kChunk;
  out->chunk = kChunk;
  hipStream_t s = ln.compute;
  const auto t_seg0 = std::chrono::steady_clock::now();   // TSG_HOST_PROFILE: where a segment's GPU time goes
  // offsets: landed with the upload (d_off_up), or copied here (resident data)
  uint64_t* d_off = const_cast<uint64_t*>(d_off_up);
  if (!d_off) {
    // staged through the lane's pinned buffer and copied by the segment
    // prologue (StageIn): a hipMemcpyAsync from the caller's pageable array
    // is a synchronous staged copy that held a resident driver thread up to
    // ~1 ms while the other driver's passes ran (r5r host timelines)
    if (!ensure(&ln.d_off, &ln.d_off_cap, in.nfiles + 1, err)) return false;
    const size_t nb = (in.nfiles + 1) * sizeof(uint64_t);
    if (ln.h_off_pin_cap[0] < in.nfiles + 1) {
      if (ln.h_off_pin[0]) hipHostFree(ln.h_off_pin[0]);
      ln.h_off_pin[0] = nullptr;
      ln.h_off_pin_cap[0] = 0;
      HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&ln.h_off_pin[0]), nb, hipHostMallocDefault));
      ln.h_off_pin_cap[0] = in.nfiles + 1;
    }
    std::memcpy(ln.h_off_pin[0], in.offsets, nb);
    void* off_dev = nullptr;
    HIP_OK(hipHostGetDevicePointer(&off_dev, ln.h_off_pin[0], 0));
    if (!off_dev || nb > 0xffffffffull) { *err = "pinned offsets staging has no device view"; return false; }
    stage.off_src = static_cast<const uint8_t*>(off_dev);
    stage.off_dst = reinterpret_cast<uint8_t*>(ln.d_off);
    stage.off_bytes = nb;
    d_off = ln.d_off;
  }
  // test hook (tsg_test_inject_segment_failures): fail here, after the
  // offsets were staged and before any launch, as a failed allocation would
  for (uint32_t k = inject_fail_.load(); k > 0;) {
    if (inject_fail_.compare_exchange_weak(k, k - 1)) { *err = "injected segment failure (test hook)"; return false; }
  }
  const size_t kw_n = static_cast<size_t>(std::max<uint32_t>(in.nfiles, 1)) * dt.kw_words;
  if (!ensure(&ln.d_kw, &ln.d_kw_cap, kw_n, err)) return false;
  const unsigned long long nchunks = (total + kChunk - 1) / kChunk;
  if (!ensure(&ln.d_nl, &ln.d_nl_cap, std::max<unsigned long long>(nchunks, 1), err)) return false;
  if (!ensure(&ln.d_cf, &ln.d_cf_cap, std::max<unsigned long long>(nchunks, 1), err)) return false;
  ln.hit_cap = std::max<size_t>(ln.hit_cap, total / 256);   // ~1 hit per 670 B on source text
  if (!ensure(&ln.d_hits, &ln.d_hits_cap, ln.hit_cap, err)) return false;
  ln.over_cap = std::max<size_t>(ln.over_cap, total / 2048);
  if (!ensure(&ln.d_over, &ln.d_over_cap, ln.over_cap, err)) return false;
  const uint32_t ngroups = static_cast<uint32_t>(dt.k1g.size());
  if (ngroups > kMaxK1Groups) { *err = "too many scan-DFA groups"; return false; }
  if (!ensure(&ln.d_bh, &ln.d_bh_cap, 2ull * std::max(dt.sms, 1) * std::max<uint32_t>(ngroups, 1), err)) return false;
  if (!ensure(&ln.d_ff, &ln.d_ff_cap, std::max<uint32_t>(in.nfiles, 1), err)) return false;
  // deferred-output slots: kOutSlots per thread (x2 grid slack)
  if (!ensure(&ln.d_ob, &ln.d_ob_cap, static_cast<size_t>(std::max(dt.sms, 1)) * 1024 * 2 * kOutSlots, err))
    return false;
  // K1's file index: entries for blocks 0 .. (total - 1) >> 16, plus one
  const uint32_t nfidx = total ? static_cast<uint32_t>(((total - 1) >> kFidxShift) + 2) : 0u;
  if (file_index_ && nfidx && !ensure(&ln.d_fidx, &ln.d_fidx_cap, nfidx, err)) return false;

  const uint32_t sms = static_cast<uint32_t>(dt.sms);
  const Prefilter& pf = pf_;
  for (int attempt = 0; attempt < 3; ++attempt) {
    constexpr uint32_t nthr = 1024;
    const uint64_t want_blocks = (nchunks + nthr - 1) / nthr;
    // one resident workgroup per CU (the LDS table takes most of the CU's
    // 160 KiB): a grid of exactly one workgroup per CU, waves take items
    // K1Chain (resident pieces): k1_reserve_cus_ CUs left out of the grid, so
    // the previous piece's K2 and readback kernels, queued behind its K1 and
    // ready while this K1 runs, find a CU at once -- K1's 1024 threads x 122
    // VGPRs fill a CU's register file, and those kernels otherwise waited for
    // the whole launch (0.8 ms per piece, profiles/r8o_*, r9d_*)
    const uint32_t reserve = chain && sms > 2 * k1_reserve_cus_ ? k1_reserve_cus_ : 0u;
    const uint32_t blocks = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(want_blocks, sms - reserve)));
    st->k1_blocks = blocks;
    st->k1_threads = nthr;
    st->table_in_lds = 1;
    // one hit region per (group, workgroup); K2 walks all of them
    const uint32_t nregions = blocks * std::max<uint32_t>(ngroups, 1);
    const uint32_t region_cap = static_cast<uint32_t>(std::min<size_t>(ln.hit_cap / nregions, 0xffffffffu));
    {
      // keyword bits, file flags, counters, per-region hit counts: one launch
      Prologue pl{};
      uint32_t* ptrs[4] = {ln.d_kw, ln.d_ff, reinterpret_cast<uint32_t*>(ln.d_cnt), ln.d_bh};
      const uint32_t ns[4] = {static_cast<uint32_t>(kw_n), std::max<uint32_t>(in.nfiles, 1),
                              static_cast<uint32_t>(kCntBytes / 4), nregions};
      uint32_t mx = 0;
      for (int k = 0; k < 4; ++k) { pl.p[k] = ptrs[k]; pl.n[k] = ns[k]; mx = std::max(mx, ns[k]); }
      uint32_t rows = 4;
      if ((stage.bytes || stage.off_bytes) && attempt == 0) {   // a small pinned batch / offsets: staged by this launch
        pl.src[0] = stage.src; pl.dst[0] = stage.dst;
        pl.bytes[0] = static_cast<uint32_t>(stage.bytes); pl.zpad[0] = stage.bytes ? 64 : 0;   // (no pad when only offsets are staged)
        pl.src[1] = stage.off_src; pl.dst[1] = stage.off_dst;
        pl.bytes[1] = static_cast<uint32_t>(stage.off_bytes); pl.zpad[1] = 0;
        mx = std::max<uint32_t>(mx, static_cast<uint32_t>(std::max(stage.bytes, stage.off_bytes) / 16 + 64));
        rows = 6;
      }
      hipLaunchKernelGGL(tsg_prologue, dim3(std::min<uint32_t>(256, (mx + 255) / 256), rows), dim3(256), 0, s, pl);
      HIP_OK(hipGetLastError());
    }
    // per-wave LDS hit buffers as large as the group's table leaves room for
    // (512 entries for the builtin rules; large config-5 groups get fewer,
    // further hits go straight to the workgroup's global region)
    auto lds_for = [&](const K1Group& g, uint32_t h) -> size_t {
      return (nthr / 64) * h * 4 + kMaxWaves * 4 + 16 + ((g.table_words16 * 2 + 15) & ~15u) + 256 + g.meta_bytes;
    };
    auto hits_of = [&](const K1Group& g) -> uint32_t {
      uint32_t h = kWaveHits;
      while (h > kK1WaveHitsMin && lds_for(g, h) > kLdsBytes) h /= 2;
      return h;
    };
    auto lds_of = [&](const K1Group& g) -> size_t { return lds_for(g, hits_of(g)); };
    for (uint32_t gi = 0; gi < ngroups; ++gi) {
      const K1Group& g = dt.k1g[gi];
      const void* kfn = k1_kernel(k1_abl_, g.compressed);
      if (!kfn) { *err = "unsupported K1 build (TSG_K1_ABL; the measurement builds are in the probe library)"; return false; }
      if (!g.in_lds || lds_of(g) > kLdsBytes) { *err = "K1 LDS budget exceeded"; return false; }
      const int want = static_cast<int>(lds_of(g));
      bool set = false;
      {
        std::lock_guard<std::mutex> lk(dt.mu);
        for (const auto& e : dt.lds_set) set = set || (e.first == kfn && e.second >= want);
      }
      if (!set) {
        HIP_OK(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, want));
        std::lock_guard<std::mutex> lk(dt.mu);
        dt.lds_set.emplace_back(kfn, want);
      }
    }
    std::unique_lock<std::mutex> chain_lk;
    if (chain && attempt == 0) {
      chain_lk = std::unique_lock<std::mutex>(chain->mu);
      if (chain->last && chain_k1_ != 2) HIP_OK(hipStreamWaitEvent(s, chain->last, 0));   // (2: no wait, K1s overlap)
    }
    HIP_OK(hipEventRecord(ln.ev[0], s));
    const uint32_t* a_fidx = nullptr;
    if (file_index_ && nfidx && nchunks > 0) {          // (inside K1's timed window)
      hipLaunchKernelGGL(tsg_file_index, dim3((nfidx + 255) / 256), dim3(256), 0, s, static_cast<const uint64_t*>(d_off),
                         in.nfiles, ln.d_fidx, nfidx);
      HIP_OK(hipGetLastError());
      a_fidx = ln.d_fidx;
    }
    uint32_t launches = 0;
    for (uint32_t gi = 0; gi < ngroups && nchunks > 0; ++gi) {
      const K1Group& g = dt.k1g[gi];
      const size_t lds = lds_of(g);
      uint32_t* a_items = ln.d_cnt + kItemCtrBase + 256 * gi;   // v3's work-item counters (zeroed with d_cnt)
      unsigned long long a_total = total;
      uint32_t a_nfiles = in.nfiles, a_ncls = g.nclasses, a_tw = g.table_words16;
      uint32_t a_first = g.first_out, a_nmeta = hits_of(g), a_nlist = g.nlist, a_nkw = pf.nkw;
      uint32_t a_warm = (k1_abl_ & kAblLine64) ? g.warm_lines64 : g.warm_lines;
      unsigned long long a_nchunks = nchunks;
      uint32_t a_chunk = kChunk;
      uint32_t a_kww = dt.kw_words, a_kwbase = g.kw_base, a_primary = gi == 0;
      const uint8_t* a_data = d_data;
      unsigned long long* a_hits = ln.d_hits + static_cast<size_t>(gi) * blocks * region_cap;
      uint32_t* a_bh = ln.d_bh + static_cast<size_t>(gi) * blocks;
      uint16_t* a_next = g.next;
      uint8_t* a_cls = g.cls;
      OutMeta* a_meta = g.meta;
      uint32_t* a_list = g.list;
      uint32_t* a_ocnt = ln.d_cnt + 2;
      uint32_t a_ocap = static_cast<uint32_t>(std::min<size_t>(ln.over_cap, 0xffffffffu));
      uint32_t a_rcap = region_cap;
      uint32_t a_tail = k1_tail_rounds_ | (top8 ? 0x100u : 0u);
      void* args[] = {&a_data, &a_total, &d_off, &a_nfiles, &a_next, &a_cls, &a_ncls, &a_tw, &a_first,
                      &a_meta, &a_nmeta, &a_list, &a_nlist, &a_nkw, &a_warm, &a_chunk, &a_nchunks,
                      &ln.d_kw, &a_kww, &a_kwbase, &a_primary, &a_hits, &a_bh, &a_rcap,
                      &ln.d_over, &a_ocnt, &a_ocap, &ln.d_nl, &ln.d_cf, &ln.d_ff, &a_items, &ln.d_ob, &a_tail,
                      &a_fidx};
      HIP_OK(hipLaunchKernel(k1_kernel(k1_abl_, g.compressed), dim3(blocks), dim3(nthr), args, lds, s));
      ++launches;
    }
    HIP_OK(hipEventRecord(ln.ev[1], s));
    st->k1_launches += launches;
    // K2 follows K1 on the stream without a host round trip: its grid is
    // sized from the lane's previous segment (or the segment's bytes), and
    // it reads the per-region hit counts and the overflow count on the
    // device; one readback + sync per segment.  An overflowed hit pool or
    // candidate buffer is seen afterwards and re-run (grown).
    bool rerun_k1 = false;
    for (int a2 = 0; a2 < 3 && !rerun_k1; ++a2) {
      if (!ensure(&ln.d_cands, &ln.d_cands_cap, ln.cand_cap, err)) return false;
      if (a2 > 0) HIP_OK(hipMemsetAsync(ln.d_cnt + 1, 0, 4, s));   // (zeroed with the counters before K1)
      // (K2's start is K1's end marker on the first attempt: a marker between
      // two kernels costs ~5 us of device time on a small segment)
      if (a2 > 0) HIP_OK(hipEventRecord(ln.ev[2], s));
      const uint64_t per_block = 256ull * k2_hits_per_thread_;
      const uint64_t maxr_est = ln.k2_maxr_per_byte > 0 ? static_cast<uint64_t>(ln.k2_maxr_per_byte * total) + 1
                                                        : 2 * (total / 2048) / nregions + 1;
      const uint32_t nsub = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(256, (maxr_est + per_block - 1) / per_block)));
      const uint32_t osub = static_cast<uint32_t>(std::max<uint64_t>(16, std::min<uint64_t>(4096, (ln.k2_over_est + 1023) / 1024)));
      const uint32_t ccap = static_cast<uint32_t>(ln.cand_cap);
      const uint32_t ocap = static_cast<uint32_t>(std::min<size_t>(ln.over_cap, 0xffffffffu));
      // the region grid, then the overflow pool's workgroups, in one launch
      const uint32_t k2_grid = nregions * nsub + osub;
      const int k2v = (ln.d_k2s ? kK2Stats : 0) | k2_abl_;
      uint32_t* k2_trace = ln.d_ob;                    // (probe builds: K1's deferred-output slots are free now)
      const void* k2fn = k2v == 0 ? reinterpret_cast<const void*>(&tsg_k2_verify<0>)
                       : k2v == kK2Stats ? reinterpret_cast<const void*>(&tsg_k2_verify<kK2Stats>)
#ifdef TSG_K1_PROBE
                       : k2v == kK2Trace ? reinterpret_cast<const void*>(&tsg_k2_verify<kK2Trace>)
                       : k2v == kK2NoWalk ? reinterpret_cast<const void*>(&tsg_k2_verify<kK2NoWalk>)
                       : k2v == (kK2Trace | kK2NoWalk) ? reinterpret_cast<const void*>(&tsg_k2_verify<kK2Trace | kK2NoWalk>)
#endif
                       : nullptr;
      if (!k2fn) { *err = "unsupported K2 build (TSG_K2_ABL: probe library only)"; return false; }
      if ((k2_abl_ & kK2Trace) && static_cast<size_t>(k2_grid) * 4 * 8 > ln.d_ob_cap / 2) { *err = "K2 trace buffer too small"; return false; }
      {
        const uint32_t a_nf = in.nfiles, a_chunk = kChunk, a_rcap = region_cap, a_nreg = nregions, a_nsub = nsub;
        const uint32_t a_ocap = ocap, a_kww = dt.kw_words, a_ccap = ccap;
        const uint8_t* a_data = d_data;
        unsigned int* a_over_cnt = ln.d_cnt + 2;
        unsigned long long a_total = total;
        void* k2args[] = {&a_data, &a_total, &d_off, const_cast<uint32_t*>(&a_nf), &ln.d_cf, const_cast<uint32_t*>(&a_chunk),
                          &ln.d_hits, &ln.d_bh, const_cast<uint32_t*>(&a_rcap), const_cast<uint32_t*>(&a_nreg),
                          const_cast<uint32_t*>(&a_nsub), &ln.d_over, &a_over_cnt, const_cast<uint32_t*>(&a_ocap),
                          &dt.anchors, &dt.rule_kw, &ln.d_kw, const_cast<uint32_t*>(&a_kww), &dt.v_next, &dt.v_cls,
                          &ln.d_cands, &ln.d_cnt, const_cast<uint32_t*>(&a_ccap), &ln.d_k2s, &k2_trace};
        HIP_OK(hipLaunchKernel(k2fn, dim3(k2_grid), dim3(256), k2args, 0, s));
      }
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(ln.ev[3], s));
      if (chain_lk.owns_lock()) {            // the other driver's next K1 follows this K2
        chain->last = chain_k1_ == 0 ? ln.ev[3] : ln.ev[1];
        chain_lk.unlock();
      }
      // (before this segment's readbacks are queued: the callback may copy
      // the lane's previous segment out of the readback buffers)
      if (while_gpu && *while_gpu) {
        (*while_gpu)();
        while_gpu = nullptr;
      }
      // everything to the host in one round trip: per-region hit counts, the
      // counters (candidates, overflow hits, LDS check), file flags, newline
      // counts and the candidates (as many as fit)
      if (!ensure_pinned(&ln.rb_bh, nregions * sizeof(uint32_t), err) || !ensure_pinned(&ln.rb_c2, 16, err) ||
          !ensure_pinned(&ln.rb_ff, in.nfiles * sizeof(uint32_t), err) ||
          !ensure_pinned(&ln.rb_nl, nchunks * sizeof(uint16_t), err) ||
          !ensure_pinned(&ln.rb_cands, ln.cand_cap * sizeof(CandDev), err)) return false;
      if (chain && readback_dma_) {
        // K1Chain: the next piece's K1 (other driver) holds every CU's
        // register file until its launch ends, so a readback kernel queued
        // behind this K2 waited for it (0.7-0.85 ms per resident piece,
        // profiles/r8o_*); copies on the DMA engines need no CU.  The
        // candidates go whole (the buffer's capacity, not the count).
        HIP_OK(hipMemcpyAsync(ln.rb_bh.p, ln.d_bh, nregions * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(ln.rb_c2.p, ln.d_cnt, 16, hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(ln.rb_ff.p, ln.d_ff, in.nfiles * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(ln.rb_nl.p, ln.d_nl, ((nchunks + 1) / 2) * 4, hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(ln.rb_cands.p, ln.d_cands, ln.cand_cap * sizeof(CandDev), hipMemcpyDeviceToHost, s));
      } else {
        Readbacks rb;
        rb.add(ln.d_bh, ln.rb_bh, nregions);
        rb.add(ln.d_cnt, ln.rb_c2, 4);
        rb.add(ln.d_ff, ln.rb_ff, in.nfiles);
        rb.add(ln.d_nl, ln.rb_nl, (nchunks + 1) / 2);
        rb.add(ln.d_cands, ln.rb_cands, ln.cand_cap * (sizeof(CandDev) / 4), ln.d_cnt + 1, sizeof(CandDev) / 4);
        if (!rb.launch(s, err)) return false;
      }
      if (chain) {
        // polled with short sleeps: a blocking-sync event woke its driver
        // 0.3-1.2 ms after the passes ended (profiles/rd5e_bench_c2prof.log)
        if (!ln.ev_sync) HIP_OK(hipEventCreateWithFlags(&ln.ev_sync, hipEventDisableTiming));
        HIP_OK(hipEventRecord(ln.ev_sync, s));
        for (;;) {
          const hipError_t q = hipEventQuery(ln.ev_sync);
          if (q == hipSuccess) break;
          if (q != hipErrorNotReady) HIP_OK(q);
          // yielding only while the confirm pool is idle: on a box whose
          // CPU share is a cgroup quota, drivers spinning beside a busy pool
          // spend the pool's quota (config 5 resident steps 16.9-20.2 ms)
          if (poll_yield_ && (!ln.pool_idle || ln.pool_idle->load(std::memory_order_relaxed))) std::this_thread::yield();
          else std::this_thread::sleep_for(std::chrono::microseconds(10));
        }
      } else {
        // (round 5 measured a host-mapped completion word written by the
        // readback's last block, spun on instead: the events' times were then
        // not yet ready and waiting for them cost a one-file batch 0.25 ms,
        // profiles/r5i_small.log; the stream synchronization stays)
        HIP_OK(hipStreamSynchronize(s));
      }
      const double t_k1_sync = ms_since(t_seg0);
      const uint32_t* h_bh = ln.rb_bh.as<const uint32_t>();
      const uint32_t* h_cnt = ln.rb_c2.as<const uint32_t>();
      if (h_cnt[3] != 0) { *err = "K1: dynamic LDS does not start at address 0"; return false; }
      float k1 = 0, k2 = 0;
      HIP_OK(hipEventElapsedTime(&k1, ln.ev[0], ln.ev[1]));
      HIP_OK(hipEventElapsedTime(&k2, a2 > 0 ? ln.ev[2] : ln.ev[1], ln.ev[3]));
      if (a2 == 0) st->k1_ms += k1;
      st->k2_ms += k2;
      const uint32_t nover = h_cnt[2];
      if (nover > ln.over_cap) {
        // the overflow pool (shared by every workgroup) was too small: grow it
        // to the exact need and run K1 again.  Growth follows the batch's
        // total hit count, not the fullest region times the region count.
        ln.over_cap = static_cast<size_t>(nover) * 5 / 4 + 1024;
        if (!ensure(&ln.d_over, &ln.d_over_cap, ln.over_cap, err)) return false;
        rerun_k1 = true;
        break;
      }
      const unsigned int c2 = h_cnt[1];
      if (c2 > ln.cand_cap) { ln.cand_cap = static_cast<size_t>(c2) * 5 / 4 + 1024; continue; }
      uint64_t nhits = 0;
      uint32_t maxr = 0;
      for (uint32_t r = 0; r < nregions; ++r) { nhits += h_bh[r]; maxr = std::max(maxr, std::min(h_bh[r], region_cap)); }
      ln.k2_maxr_per_byte = total ? static_cast<double>(maxr) * 1.25 / static_cast<double>(total) : 0.0;
      ln.k2_over_est = nover;
      st->hits += nhits;
      auto t_d2h = std::chrono::steady_clock::now();
      out->rb_cands = ln.rb_cands.as<CandDev>();
      out->rb_ff = ln.rb_ff.as<uint32_t>();
      out->rb_nl = ln.rb_nl.as<uint16_t>();
      out->n_cands = c2;
      out->n_ff = in.nfiles;
      out->n_nl = nchunks;
      out->deferred = true;
      if (!defer_copy) out->finish_copy();
      st->d2h_ms += ms_since(t_d2h);
      if (host_profile_)
        std::fprintf(stderr, "[tsg seg] %.1f MB %u files: wall to results %.3f ms (K1 %.3f, K2 %.3f, K2 grid %u+%u), "
                     "copy-out %.3f ms, total %.3f ms\n", total / 1e6, in.nfiles, t_k1_sync, k1, k2, nregions * nsub,
                     osub, ms_since(t_d2h), ms_since(t_seg0));
      st->candidates += c2;
#ifdef TSG_K1_PROBE
      if (k2_abl_ & kK2Trace) {
        // probe builds: K2's per-wave stamps appended to $TSG_K2_TRACE_FILE as
        // [waves, 0, 0, 0][8 x waves] uint32
        const size_t waves = static_cast<size_t>(k2_grid) * 4;
        std::vector<uint32_t> tr(4 + 8 * waves, 0);
        tr[0] = static_cast<uint32_t>(waves);
        HIP_OK(hipMemcpy(tr.data() + 4, k2_trace, 8 * waves * sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (const char* fn = std::getenv("TSG_K2_TRACE_FILE")) {
          if (FILE* fp = std::fopen(fn, "ab")) {
            std::fwrite(tr.data(), sizeof(uint32_t), tr.size(), fp);
            std::fclose(fp);
          }
        }
      }
      if (k1_abl_ & kAblTrace) {
        // probe builds: the K1 launch's stamps (kAblTrace) appended to
        // $TSG_K1_TRACE_FILE as [blocks, items, nchunks, chunk][4 x blocks][kTraceItemWords x items] uint32
        const uint32_t items = static_cast<uint32_t>(std::min<uint64_t>(kTraceItemCap, 3 * (nchunks + 63) / 64 + 64));
        std::vector<uint32_t> tr(4 + 4 * static_cast<size_t>(blocks) + kTraceItemWords * static_cast<size_t>(items), 0);
        tr[0] = blocks; tr[1] = items; tr[2] = static_cast<uint32_t>(nchunks); tr[3] = kChunk;
        HIP_OK(hipMemcpy(tr.data() + 4, ln.d_ob + static_cast<size_t>(blocks) * nthr * kOutSlots,
                         (tr.size() - 4) * sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (const char* fn = std::getenv("TSG_K1_TRACE_FILE")) {
          if (FILE* fp = std::fopen(fn, "ab")) {
            std::fwrite(tr.data(), sizeof(uint32_t), tr.size(), fp);
            std::fclose(fp);
          }
        }
        HIP_OK(hipMemset(ln.d_ob + static_cast<size_t>(blocks) * nthr * kOutSlots, 0, (tr.size() - 4) * sizeof(uint32_t)));
      }
#endif
      if (ln.d_k2s) {
        std::vector<unsigned long long> h(kK2Stat * pf_.rules.size());
        HIP_OK(hipMemcpy(h.data(), ln.d_k2s, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        HIP_OK(hipMemset(ln.d_k2s, 0, h.size() * sizeof(unsigned long long)));
        std::lock_guard<std::mutex> lk(k2s_mu_);
        if (k2s_.size() < h.size()) k2s_.resize(h.size(), 0);
        for (size_t i = 0; i < h.size(); ++i)
          k2s_[i] = i % kK2Stat == 4 ? std::max(k2s_[i], h[i]) : k2s_[i] + h[i];
      }
      return true;
    }
    if (rerun_k1) continue;
    *err = "candidate buffer overflow persisted";
    return false;
  }
  *err = "hit buffer overflow persisted";
  return false;
}

bool Engine::prefilter_only(const BatchInput& in, std::vector<std::vector<std::vector<uint64_t>>>* cands,
                            ScanStats* st, std::string* err) {
  ScanStats local;
  if (!st) st = &local;
  if (!in.d_data) { *err = "prefilter_only needs device-resident data"; return false; }
  DeviceTables& dt = *dev_[0];
  Lane* ln = acquire_lane(dt, err);
  if (!ln) return false;
  Segment sg;
  sg.in = in;
  GpuOut out;
  const bool ok = run_segment(dt, *ln, sg, in.d_data, nullptr, st, &out, err);
  release_lane(dt, ln);
  if (!ok) return false;
  const size_t nr = rs_->rules.size();   // real rules only (exclude pseudo-rules follow)
  if (cands) {
    cands->assign(in.nfiles, std::vector<std::vector<uint64_t>>(nr));
    for (const CandDev& c : out.cands)
      if (c.rule < nr) (*cands)[c.file][c.rule].push_back(c.start);
    for (auto& f : *cands)
      for (auto& v : f) { std::sort(v.begin(), v.end()); v.erase(std::unique(v.begin(), v.end()), v.end()); }
  }
  return true;
}

bool Engine::feed_probe(const uint8_t* h_data, uint64_t bytes, double* ms, std::string* err) {
  DeviceTables& dt = *dev_[0];
  Lane* ln = acquire_lane(dt, err);
  if (!ln) return false;
  bool ok = hipSetDevice(dt.device) == hipSuccess;
  const uint64_t seg = std::min<uint64_t>(segment_, std::max<uint64_t>(bytes, 1));
  for (int i = 0; i < 2 && ok; ++i) ok = ensure(&ln->ring[i], &ln->ring_cap[i], seg + 64, err);
  auto t0 = std::chrono::steady_clock::now();
  int slot = 0;
  for (uint64_t o = 0; ok && o < bytes; o += seg, slot ^= 1) {
    const uint64_t n = std::min(seg, bytes - o);
    ok = hipMemcpyAsync(ln->ring[slot], h_data + o, n, hipMemcpyHostToDevice, ln->copy) == hipSuccess;
  }
  ok = ok && hipStreamSynchronize(ln->copy) == hipSuccess;
  *ms = ms_since(t0);
  release_lane(dt, ln);
  if (!ok && err->empty()) *err = "feed probe copy failed";
  return ok;
}

bool Engine::strip_cr(const void* d_src, const uint64_t* d_off, uint32_t nfiles, uint64_t total, void* d_dst,
                      uint64_t* d_new_off, uint64_t* out_total, double* ms, std::string* err) {
  if ((reinterpret_cast<uintptr_t>(d_src) | reinterpret_cast<uintptr_t>(d_dst)) & 15u) {
    *err = "CR strip buffers must be 16-byte aligned";
    return false;
  }
  if (!d_off || !d_new_off || (total && (!d_src || !d_dst))) { *err = "CR strip: null buffer"; return false; }
  // every buffer must be memory of one device the engine spans; the kernels
  // run there (an engine over several devices takes the caller's device)
  const int dev = device_of(d_off);
  DeviceTables* dtp = nullptr;
  for (auto& d : dev_) if (d->device == dev) { dtp = d.get(); break; }
  if (!dtp || device_of(d_new_off) != dev || (total && (device_of(d_src) != dev || device_of(d_dst) != dev))) {
    *err = "CR strip buffers must be device memory of one of the engine's devices";
    return false;
  }
  DeviceTables& dt = *dtp;
  Lane* ln = acquire_lane(dt, err);
  if (!ln) return false;
  bool ok = hipSetDevice(dt.device) == hipSuccess;
  uint64_t ends[2] = {1, 0};
  ok = ok && hipMemcpyAsync(&ends[0], d_off, 8, hipMemcpyDeviceToHost, ln->compute) == hipSuccess &&
       hipMemcpyAsync(&ends[1], d_off + nfiles, 8, hipMemcpyDeviceToHost, ln->compute) == hipSuccess &&
       hipStreamSynchronize(ln->compute) == hipSuccess;
  if (ok && (ends[0] != 0 || ends[1] != total)) {
    *err = "CR strip: offsets must run from 0 to the batch size";
    ok = false;
  }
  ok = ok && ensure(&ln->d_cr, &ln->d_cr_cap, cr_strip_scratch_bytes(total), err);
  ok = ok && hipEventRecord(ln->ev[0], ln->compute) == hipSuccess;
  ok = ok && cr_strip_launch(static_cast<const uint8_t*>(d_src), d_off, nfiles, total, static_cast<uint8_t*>(d_dst),
                             d_new_off, ln->d_cr, ln->compute, err);
  ok = ok && hipEventRecord(ln->ev[1], ln->compute) == hipSuccess;
  uint64_t stripped = 0;
  ok = ok && hipMemcpyAsync(&stripped, ln->d_cr, 8, hipMemcpyDeviceToHost, ln->compute) == hipSuccess &&
       hipStreamSynchronize(ln->compute) == hipSuccess;
  float kms = 0;
  if (ok && ms) ok = hipEventElapsedTime(&kms, ln->ev[0], ln->ev[1]) == hipSuccess;
  release_lane(dt, ln);
  if (!ok) {
    if (err->empty()) *err = "CR strip failed on the device";
    return false;
  }
  if (out_total) *out_total = stripped;
  if (ms) *ms = kms;
  return true;
}

// Host confirmation of one segment (files [0, in.nfiles) of sg.in, results
// into results[0..nfiles)) from that segment's GPU output `g`.
void Engine::plan_confirm(const Segment& sg, GpuOut* gp) const {
  GpuOut& g = *gp;
  const BatchInput& in = sg.in;
  const size_t nr = rs_->rules.size();
  // group candidates per file (counting sort by file, then sort each file's list)
  g.per_file.assign(in.nfiles + 1, 0);
  for (const CandDev& c : g.cands) g.per_file[c.file + 1]++;
  for (uint32_t f = 0; f < in.nfiles; ++f) g.per_file[f + 1] += g.per_file[f];
  g.sorted.resize(g.cands.size());
  {
    std::vector<uint32_t> pos(g.per_file.begin(), g.per_file.end() - 1);
    for (const CandDev& c : g.cands) g.sorted[pos[c.file]++] = c;
  }
  bool any_full = false;
  for (size_t r = 0; r < nr; ++r) if (pf_.rules[r].mode == 1) any_full = true;
  // files to confirm (candidates, fold-special content, or host-evaluated
  // rules), largest first (LPT: the per-file confirm cost grows with size);
  // every other file only needs the global allow-path outcome and is handled
  // in blocks after them (image layers: hundreds of thousands of such files)
  g.work.clear();
  g.light.clear();
  g.work.reserve(in.nfiles / 4 + 16);
  for (uint32_t f = sg.lead; f < in.nfiles; ++f) {
    if (any_full || g.ff[f] || g.per_file[f] != g.per_file[f + 1]) g.work.push_back(f);
    else g.light.push_back(f);
  }
  // largest first, by power-of-two size class (a counting sort: a full sort
  // of config 5's 13k files per piece cost ~1 ms on the confirming thread;
  // LPT within a factor of two balances the pool as well)
  {
    uint32_t cnt[65] = {};
    auto cls = [&](uint32_t f) {
      const uint64_t n = in.offsets[f + 1] - in.offsets[f];
      return 63 - __builtin_clzll(n + 1);           // 0..63
    };
    for (uint32_t f : g.work) ++cnt[63 - cls(f) + 1];
    for (int k = 1; k <= 64; ++k) cnt[k] += cnt[k - 1];
    std::vector<uint32_t> by(g.work.size());
    for (uint32_t f : g.work) by[cnt[63 - cls(f)]++] = f;
    g.work.swap(by);
  }
  g.planned = true;
}

void Engine::confirm_segment(CallCtx& cc, const Segment& sg, GpuOut& g, Secret* results, uint64_t* nconf_out,
                             uint64_t* nfind_out, bool gpu_in_flight) {
  const BatchInput& in = sg.in;
  const Ruleset& rs = *rs_;
  const size_t nplan = pf_.rules.size();   // rules + exclude-block pseudo-rules
  const auto t_begin = std::chrono::steady_clock::now();
  if (!g.planned) plan_confirm(sg, &g);
  const std::vector<uint32_t>& per_file = g.per_file;
  std::vector<CandDev>& sorted = g.sorted;
  const std::vector<uint32_t>& work = g.work;
  const std::vector<uint32_t>& light = g.light;
  // the plan every confirmed file starts from, and its mode-1 rules
  std::vector<uint8_t> kind0(nplan, kPlanNoMatch);
  std::vector<uint32_t> full_rules;
  for (size_t r = 0; r < nplan; ++r) {
    if (pf_.rules[r].mode == 1) {            // (mode 3: only with a presence candidate)
      kind0[r] = kPlanFull;
      full_rules.push_back(static_cast<uint32_t>(r));
    }
  }
  results -= sg.lead;                      // results[f] for the piece's files f >= lead
  constexpr uint32_t kLightBlock = 512;
  const uint32_t nlight_blocks = static_cast<uint32_t>((light.size() + kLightBlock - 1) / kLightBlock);
  std::atomic<uint32_t> next_light{0};
  std::atomic<uint32_t> next{0};
  std::atomic<uint64_t> nfind{0}, nconf{0};
  // TSG_HOST_PROFILE: worker thread-ns in the plan (candidates sorted and
  // grouped), scan_file and storing the result
  std::atomic<uint64_t> ph_plan{0}, ph_scan{0}, ph_store{0};
  const bool prof = host_profile_;
  auto light_files = [&]() {
    for (;;) {
      const uint32_t b = next_light.fetch_add(1);
      if (b >= nlight_blocks) break;
      const size_t e = std::min<size_t>(light.size(), (static_cast<size_t>(b) + 1) * kLightBlock);
      for (size_t k = static_cast<size_t>(b) * kLightBlock; k < e; ++k) {
        const uint32_t f = light[k];
        if (confirm_prefetch_ && k + 8 < e) __builtin_prefetch(in.paths[light[k + 8]]);   // (path strings: scattered)
        // no candidates, no host-evaluated rule: only the global allow-path outcome remains
        const char* p = in.paths[f];
        const size_t pn = in.path_lens ? in.path_lens[f] : std::strlen(p);
        if (global_allow_path(rs, reinterpret_cast<const uint8_t*>(p), pn)) results[f] = Secret::path_only(p, pn);
      }
    }
  };
  auto worker = [&]() {
    FilePlan plan;
    std::vector<std::vector<uint64_t>> spare;
    // per-thread counts and work taken a few files at a time: 15 threads
    // hitting shared counters once per file serialised on their cache lines
    uint64_t my_conf = 0, my_find = 0, my_plan = 0, my_scan = 0, my_store = 0;
    constexpr uint32_t kTake = 4;
    uint32_t wi = 0, wend = 0;
    for (;;) {
      if (wi == wend) {
        wi = next.fetch_add(kTake);
        if (wi >= work.size()) break;
        wend = std::min<uint32_t>(wi + kTake, static_cast<uint32_t>(work.size()));
      }
      uint32_t f = work[wi++];
      if (confirm_prefetch_ && wi < wend) {
        // the next file of this take: its result slot and the text at its
        // first candidate starts, fetched while this file is confirmed (the
        // host has not touched the batch's bytes since they were written):
        // resident config 5 602-611 -> 614-657 GB/s (profiles/r6j_confirm_prefetch_c5.log; two files
        // ahead and a wider window were no better)
        const uint32_t fn = work[wi];
        __builtin_prefetch(results + fn, 1);
        __builtin_prefetch(in.paths[fn]);
        const uint8_t* cn = in.h_data + in.offsets[fn];
        const uint64_t ln = in.offsets[fn + 1] - in.offsets[fn];
        for (uint32_t k = per_file[fn], ke = std::min(per_file[fn + 1], per_file[fn] + 4); k < ke; ++k) {
          const uint64_t st = sorted[k].start;
          if (st < ln) {
            __builtin_prefetch(cn + st);
            if (st + 64 < ln) __builtin_prefetch(cn + st + 64);
          }
        }
      }
      const auto tp0 = prof ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
      const char* path_p = in.paths[f];
      const size_t path_n = in.path_lens ? in.path_lens[f] : std::strlen(path_p);
      const uint8_t* content = in.h_data + in.offsets[f];
      const size_t len = in.offsets[f + 1] - in.offsets[f];
      const bool binary = in.binary ? in.binary[f] != 0 : false;
      const uint32_t cb = per_file[f], ce = per_file[f + 1];
      if (g.ff[f]) {
        // fold-special file (U+0130/U+212A/U+017F present): the two passes run
        // on the host with the variant scan DFA, then the exact confirmer
        ++my_conf;
        std::vector<std::vector<uint64_t>> vc;
        std::vector<uint8_t> vg;
        prefilter_variant_file(pf_, content, len, &vc, &vg);
        plan_from_candidates(pf_, &vc, &plan);
        Secret s = scan_file(rs, path_p, path_n, content, len, binary, &plan);
        my_find += s.findings().size();
        results[f] = std::move(s);
        continue;
      }
      ++my_conf;
      plan.kind = kind0;                       // mode-1 rules kPlanFull, the rest kPlanNoMatch
      for (RuleCandidates& c : plan.cands) {   // start lists are reused from file to file
        c.starts.clear();
        spare.push_back(std::move(c.starts));
      }
      plan.cands.clear();
      std::sort(sorted.begin() + cb, sorted.begin() + ce, [](const CandDev& a, const CandDev& b) {
        return a.rule != b.rule ? a.rule < b.rule : a.start < b.start;
      });
      for (uint32_t k = cb; k < ce;) {
        uint32_t r = sorted[k].rule;
        RuleCandidates rc;
        rc.rule = r;
        if (!spare.empty()) {
          rc.starts = std::move(spare.back());
          spare.pop_back();
        }
        while (k < ce && sorted[k].rule == r) {
          if (rc.starts.empty() || rc.starts.back() != sorted[k].start) rc.starts.push_back(sorted[k].start);
          ++k;
        }
        // mode 3 presence candidates, and a mode-4 walk that gave up
        // (kFullScanStart sorts last): the rule in full on the host
        plan.kind[r] = pf_.rules[r].mode == 3 || rc.starts.back() == kFullScanStart ? kPlanFull
                     : pf_.rules[r].gate_on_gpu ? kPlanCandidates : kPlanCandHostGate;
        plan.cands.push_back(std::move(rc));
      }
      // the rules scan_file visits: mode-1 rules and those with candidates, ascending
      plan.active.clear();
      plan.active_set = true;
      {
        size_t a = 0, b = 0;
        while (a < full_rules.size() || b < plan.cands.size()) {
          const uint32_t x = a < full_rules.size() ? full_rules[a] : UINT32_MAX;
          const uint32_t y = b < plan.cands.size() ? plan.cands[b].rule : UINT32_MAX;
          if (x <= y) { plan.active.push_back(x); ++a; if (x == y) ++b; }
          else { plan.active.push_back(y); ++b; }
        }
      }
      NlSource nls;
      nls.chunk_nl = g.nl.data();
      nls.data = in.h_data;
      nls.file_off = in.offsets[f];
      nls.chunk = g.chunk;
      const auto tp1 = prof ? std::chrono::steady_clock::now() : tp0;
      Secret s = scan_file(rs, path_p, path_n, content, len, binary, &plan, &nls);
      const auto tp2 = prof ? std::chrono::steady_clock::now() : tp0;
      my_find += s.findings().size();
      results[f] = std::move(s);
      if (prof) {
        const auto tp3 = std::chrono::steady_clock::now();
        my_plan += std::chrono::duration_cast<std::chrono::nanoseconds>(tp1 - tp0).count();
        my_scan += std::chrono::duration_cast<std::chrono::nanoseconds>(tp2 - tp1).count();
        my_store += std::chrono::duration_cast<std::chrono::nanoseconds>(tp3 - tp2).count();
      }
    }
    nconf.fetch_add(my_conf);
    nfind.fetch_add(my_find);
    if (prof) { ph_plan += my_plan; ph_scan += my_scan; ph_store += my_store; }
  };
  // small confirmations (a few files, little text: per-file Scan batches) run
  // on this thread; waking the pool costs more than the work
  uint64_t work_bytes = 0;
  for (size_t k = 0; k < work.size() && work_bytes <= kInlineConfirmBytes; ++k)
    work_bytes += in.offsets[work[k] + 1] - in.offsets[work[k]];
  const bool inline_confirm = work.size() <= kInlineConfirmFiles && work_bytes <= kInlineConfirmBytes &&
                              light.size() <= kLightBlock;
  const int nt = inline_confirm ? 1 : cc.get().size();
  // while GPU passes are in flight one core stays with each thread driving
  // them (a preempted driver thread stalls its GPU)
  const int active = gpu_in_flight && nt > 1 ? nt - 1 : nt;
  const double t_setup = ms_since(t_begin);
  std::atomic<uint64_t> work_us{0}, light_us{0};
  auto body = [&](int idx) {
    if (idx >= active) return;
    auto a = std::chrono::steady_clock::now();
    worker();
    auto b = std::chrono::steady_clock::now();
    light_files();
    work_us.fetch_add(std::chrono::duration_cast<std::chrono::microseconds>(b - a).count());
    light_us.fetch_add(std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - b).count());
  };
  if (inline_confirm) body(0);
  else cc.get().run(body);
  if (host_profile_) {
    uint64_t ph[5];
    for (int k = 0; k < 5; ++k) ph[k] = g_scan_prof[k].exchange(0);
    std::fprintf(stderr, "[tsg host] files %u (work %zu, light %zu) cands %zu: setup %.2f ms, wall %.2f ms, "
                 "work %.1f + light %.1f thread-ms on %d threads (plan %.1f, scan_file %.1f, store %.1f); scan_file "
                 "thread-ms: keywords %.1f, find %.1f, blocks %.1f, findings %.1f, sort %.1f\n", in.nfiles,
                 work.size(), light.size(), g.cands.size(), t_setup, ms_since(t_begin), work_us.load() / 1e3,
                 light_us.load() / 1e3, active, ph_plan.load() / 1e6, ph_scan.load() / 1e6, ph_store.load() / 1e6,
                 ph[0] / 1e6, ph[1] / 1e6, ph[2] / 1e6, ph[3] / 1e6, ph[4] / 1e6);
  }
  *nconf_out += nconf.load();
  *nfind_out += nfind.load();
}

// One batch through the pipeline:
//  * uploaded data (h_data only): the batch is cut into segments of about
//    segment_ bytes at file boundaries; each device's driver thread takes
//    segments from a shared queue, uploads the next one on its copy stream
//    while K1/K2 of the current one run on its compute stream (two-slot
//    upload ring), and hands each finished segment to this thread, which
//    confirms it on the host while the drivers go on;
//  * resident data (d_data on one of the engine's devices): pieces (TSG_PIECES,
//    the first taking first_piece_ of the bytes), GPU passes of piece i+1 on
//    the driver while this thread confirms piece i.
// Every segment is a self-contained batch (offsets rebased to 0, data a
// 16-byte aligned sub-range), so the kernels are unchanged and the result is
// the one-segment result.
bool Engine::scan(const BatchInput& in, SecretVec* results, ScanStats* st, std::string* err) {
  ScanStats local;
  if (!st) st = &local;
  *st = ScanStats();
  auto t0 = std::chrono::steady_clock::now();
  if (in.nfiles && !in.offsets) { *err = "offsets is NULL"; return false; }
  if (in.offsets && in.offsets[0] != 0) { *err = "offsets[0] must be 0"; return false; }
  for (uint32_t i = 0; i < in.nfiles; ++i) {
    if (in.offsets[i + 1] < in.offsets[i]) { *err = "offsets must be non-decreasing"; return false; }
  }
  const uint64_t total = in.nfiles ? in.offsets[in.nfiles] : 0;
  st->bytes = total;
  st->files = in.nfiles;
  if (in.nfiles == 0 || total == 0) {
    // nothing for the GPU: every file is empty, so only the global
    // allow-path outcome (scanner.go:381-386) can make a Secret non-empty
    results->clear();
    results->resize(in.nfiles);
    for (uint32_t f = 0; f < in.nfiles; ++f)
      (*results)[f] = scan_file(*rs_, in.path_lens ? std::string(in.paths[f], in.path_lens[f]) : std::string(in.paths[f]),
                                in.h_data, 0, in.binary ? in.binary[f] != 0 : false, nullptr);
    st->pieces = 0;
    st->total_ms = ms_since(t0);
    return true;
  }
  // --- segments
  std::vector<Segment> segs;
  std::vector<DeviceTables*> drivers;
  const bool resident = in.d_data != nullptr;
  {
    std::vector<uint32_t> cut{0};
    if (resident) {
      const int dev = device_of(in.d_data);
      for (auto& d : dev_) if (d->device == dev) { drivers.push_back(d.get()); break; }
      if (drivers.empty()) { *err = "d_data is not device memory of one of the engine's devices"; return false; }
      const uint32_t want = static_cast<uint32_t>(std::min<uint64_t>(pieces_, std::max<uint64_t>(1, total / min_piece_)));
      // piece 0 takes first_piece_ of the bytes; with last_piece_ a short
      // last piece of that share follows the others (its confirmation is the
      // tail left after the GPU's last pass); the rest share what remains
      const bool short_last = last_piece_ > 0.0 && want >= 5;
      // batches of 3 pieces (0.75-1 GB) start with a larger piece
      // (TSG_FIRST_PIECE_FEW; 1 GB of config-1 files: 1.49-1.50 ms per step
      // at 10%, 1.43-1.46 at 20%, 1.45-1.46 at 30%, profiles/r8d_*)
      const double first = want == 3 ? first_piece_few_ : first_piece_;
      const double mid = 1.0 - first - (short_last ? last_piece_ : 0.0);
      const uint32_t nmid = want - 1 - (short_last ? 1 : 0);
      for (uint32_t p = 1; p < want; ++p) {
        const double share = p <= nmid ? first + mid * (p - 1) / nmid : 1.0 - last_piece_;
        const uint64_t target = static_cast<uint64_t>(share * static_cast<double>(total));
        const uint32_t f = static_cast<uint32_t>(std::lower_bound(in.offsets, in.offsets + in.nfiles, target) - in.offsets);
        if (f > cut.back() && f < in.nfiles) cut.push_back(f);
      }
    } else {
      // Geometric tail: the work left after the last upload is the last
      // segment's K1/K2 and host confirmation.  For batches whose confirm
      // cost per byte is high (many small files: image layers, config 5) or
      // that are too small for several full segments, the rest after the full
      // segments is cut in halves down to segment_min_, so the last segment
      // is small and every upload overlaps the previous segment's work.
      // Large-file batches keep full segments (K1 runs at its large-launch
      // rate and their confirmation is cheap).
      const bool dense = static_cast<double>(in.nfiles) * 1e9 > kDenseFilesPerGB * static_cast<double>(total);
      const bool geometric = dense || total < 2 * segment_;
      for (uint32_t f = 0; f < in.nfiles;) {
        // next cut: the first file boundary at or past segment_ bytes from
        // here; optionally (segment_tail_ > 0) the batch ends in a short
        // segment, so the kernels and confirmation left after the last upload
        // are shorter (measured: ~1 ms of a 179 ms 10 GB step, while the
        // short launch runs K1 at ~2.1 TB/s against 3 TB/s for 4 GB)
        const uint64_t rest = total - in.offsets[f];
        const uint64_t tail = std::min(segment_tail_, segment_ / 8);
        uint64_t target;
        // (geometric batches start halving once less than two full segments
        // are left: a full segment's confirmation then hides behind the next
        // half-size upload; r3t config 5: 4.3+4.3+0.7+... GB left 16 ms after
        // the last upload, the second segment's 25 ms confirmation)
        // (large-file batches: the rest is cut into ceil(rest / segment_)
        // equal segments instead of full segments plus a short remainder, so
        // every K1 launch runs at its large-launch rate: a 10 GB batch is
        // 3 x 3.33 GB, not 4 + 4 + 1.4 GB whose last launch ran at ~2.3 TB/s;
        // TSG_SEGMENT_BALANCED=0 keeps full segments)
        const uint64_t kleft = (rest + segment_ - 1) / segment_;
        if (!geometric && balanced_ && tail == 0 && kleft >= 2) target = in.offsets[f] + rest / kleft;
        else if (geometric ? rest >= 2 * segment_ : rest > segment_ + tail) target = in.offsets[f] + segment_;
        else if (geometric && rest / 2 >= segment_min_) target = in.offsets[f] + rest / 2;
        else if (tail > 0 && rest > 2 * tail) target = total - tail;
        else break;
        uint32_t g = static_cast<uint32_t>(std::lower_bound(in.offsets + f, in.offsets + in.nfiles, target) - in.offsets);
        if (g <= f) g = f + 1;
        if (g >= in.nfiles) break;
        cut.push_back(g);
        f = g;
      }
      const size_t nseg = cut.size();
      for (auto& d : dev_) {
        if (drivers.size() >= nseg) break;
        drivers.push_back(d.get());
      }
    }
    cut.push_back(in.nfiles);
    segs.resize(cut.size() - 1);
    for (size_t p = 0; p < segs.size(); ++p) {
      const uint32_t a = cut[p], b = cut[p + 1];
      Segment& sg = segs[p];
      BatchInput& q = sg.in;
      q = in;
      sg.f0 = a;
      sg.b0 = in.offsets[a];
      sg.bytes = in.offsets[b] - in.offsets[a];
      if (segs.size() > 1) {
        sg.off.resize(b - a + 1);
        for (uint32_t f = a; f <= b; ++f) sg.off[f - a] = in.offsets[f] - sg.b0;
        q.offsets = sg.off.data();
      }
      q.nfiles = b - a;
      q.h_data = in.h_data ? in.h_data + sg.b0 : nullptr;
      q.d_data = resident ? static_cast<const uint8_t*>(in.d_data) + sg.b0 : nullptr;
      q.paths = in.paths ? in.paths + a : nullptr;
      q.path_lens = in.path_lens ? in.path_lens + a : nullptr;
      q.binary = in.binary ? in.binary + a : nullptr;
      // a resident piece after the first starts at an arbitrary file offset:
      // K1 reads 64-byte lines from the piece's base, and a base off the
      // 128-byte L2 line grid made it fetch 2.4 HBM bytes per content byte
      // (aligned pieces 1.5, profiles/rd4k traffic runs).  Start it at the
      // 256-byte boundary below, the bytes in between a lead file.
      const uint64_t delta = resident && p > 0 ? (reinterpret_cast<uintptr_t>(in.d_data) + sg.b0) & 255u : 0;
      if (delta && in.h_data && in.paths) {
        sg.lead = 1;
        sg.off.insert(sg.off.begin(), 0);
        for (size_t k = 1; k < sg.off.size(); ++k) sg.off[k] += delta;
        q.offsets = sg.off.data();
        q.nfiles = b - a + 1;
        q.h_data -= delta;
        q.d_data = static_cast<const uint8_t*>(q.d_data) - delta;
        sg.lead_paths.assign(1, "");
        sg.lead_paths.insert(sg.lead_paths.end(), in.paths + a, in.paths + b);
        q.paths = sg.lead_paths.data();
        if (in.path_lens) {
          sg.lead_lens.assign(1, 0);
          sg.lead_lens.insert(sg.lead_lens.end(), in.path_lens + a, in.path_lens + b);
          q.path_lens = sg.lead_lens.data();
        }
        if (in.binary) {
          sg.lead_bin.assign(1, 0);
          sg.lead_bin.insert(sg.lead_bin.end(), in.binary + a, in.binary + b);
          q.binary = sg.lead_bin.data();
        }
      }
    }
  }
  // resident batches of several pieces: two drivers on the device (K1Chain)
  const bool dual = resident && segs.size() >= 2 && resident_drivers_ >= 2;
  K1Chain chain;
  K1Chain* chain_p = dual ? &chain : nullptr;
  if (dual) drivers.push_back(drivers[0]);
  uint64_t max_seg = 0;
  size_t max_seg_files = 0;
  for (const Segment& sg : segs) {
    max_seg = std::max(max_seg, sg.bytes);
    max_seg_files = std::max<size_t>(max_seg_files, sg.in.nfiles);
  }

  struct Job {
    size_t seg = 0;
    GpuOut out;
  };
  // the segment counter, the job queue and the driver fan-out (pipeline.h;
  // its failure behaviour is tested on simulated devices by
  // tsg_test_multi_driver_model)
  DriverPipeline<Job> pipe(static_cast<int>(drivers.size()), segs.size());
  JobQueue<Job>& q = pipe.queue();
  std::mutex st_mu;
  double gpu_busy = 0;
  auto t_feed0 = std::chrono::steady_clock::now();
  std::atomic<int64_t> feed_end_ns{0};
  std::atomic<bool> confirmer_idle{true};
  // a batch small enough for one segment in pinned host memory: staged by the
  // segment prologue over PCIe (tsg_prologue) instead of the copy engine
  const uint8_t* h_dev = nullptr;
  if (!resident && segs.size() == 1 && drivers.size() == 1 && total <= kDirectStageBytes && in.h_data) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, in.h_data) == hipSuccess && a.type == hipMemoryTypeHost && a.devicePointer) {
      // (the attributes may describe the allocation's base: offset the device view likewise)
      const uint8_t* hp = a.hostPointer ? static_cast<const uint8_t*>(a.hostPointer) : in.h_data;
      h_dev = static_cast<const uint8_t*>(a.devicePointer) + (in.h_data - hp);
    } else

      (void)hipGetLastError();
  }
  const bool direct = h_dev != nullptr;
  auto driver = [&](int di, std::string* e_out) -> bool {
    DeviceTables* dt = drivers[di];
    std::string e;
    ScanStats dst;
    auto tb = std::chrono::steady_clock::now();
    Lane* ln = nullptr;
    bool ok = false;
    // (a host exception -- bad_alloc of a plan or a copy-out -- ends this
    // driver like a HIP error: the queue is aborted and the call fails; it
    // must not escape the thread)
    try {
    ln = acquire_lane(*dt, &e);
    ok = ln != nullptr;
    if (ok) ln->pool_idle = &confirmer_idle;
    if (ok && hipSetDevice(dt->device) != hipSuccess) { ok = false; e = "hipSetDevice failed"; }
    if (ok && !resident) {
      for (int i = 0; i < 2 && ok; ++i) {
        ok = ensure(&ln->ring[i], &ln->ring_cap[i], max_seg + 64, &e) &&
             ensure(&ln->off_slot[i], &ln->off_slot_cap[i], max_seg_files + 1, &e);
        if (ok && ln->h_off_pin_cap[i] < max_seg_files + 1) {
          if (ln->h_off_pin[i]) hipHostFree(ln->h_off_pin[i]);
          ln->h_off_pin[i] = nullptr;
          ln->h_off_pin_cap[i] = 0;
          if (hipHostMalloc(reinterpret_cast<void**>(&ln->h_off_pin[i]), (max_seg_files + 1) * sizeof(uint64_t),
                            hipHostMallocDefault) != hipSuccess) { ok = false; e = "pinned offsets staging"; }
          else ln->h_off_pin_cap[i] = max_seg_files + 1;
        }
      }
    }
    // upload of segment `si` into ring slot `slot` (copy stream)
    auto upload = [&](size_t si, int slot) -> bool {
      const Segment& sg = segs[si];
      std::string* err = &e;
      HIP_OK(hipEventRecord(ln->up_begin[slot], ln->copy));
      // the slot's staging was last read by the upload two segments back,
      // complete since that segment's kernels waited on it
      std::memcpy(ln->h_off_pin[slot], sg.in.offsets, (sg.in.nfiles + 1) * sizeof(uint64_t));
      HIP_OK(hipMemcpyAsync(ln->off_slot[slot], ln->h_off_pin[slot], (sg.in.nfiles + 1) * sizeof(uint64_t),
                            hipMemcpyHostToDevice, ln->copy));
      HIP_OK(hipMemcpyAsync(ln->ring[slot], sg.in.h_data, sg.bytes, hipMemcpyHostToDevice, ln->copy));
      HIP_OK(hipMemsetAsync(ln->ring[slot] + sg.bytes, 0, 64, ln->copy));   // K1 reads 16-B words past the end
      HIP_OK(hipEventRecord(ln->up_done[slot], ln->copy));
      return true;
    };
    // a finished segment is handed to the confirmer once this thread has
    // queued the next segment's kernels and planned its confirmation
    // (plan_confirm) while they run: the confirming pool never waits on the
    // plan of a segment whose successor is on the GPU
    // (an idle confirmer gets the segment at once and plans it itself)
    std::unique_ptr<Job> pending;
    const std::function<void()> plan_pending = [&]() {
      if (!pending) return;
      pending->out.finish_copy();
      if (!confirmer_idle.load(std::memory_order_acquire)) plan_confirm(segs[pending->seg], &pending->out);
      q.push(std::move(pending));
    };
    size_t cur = ok ? pipe.next_segment() : segs.size();
    int slot = 0;
    if (ok && host_profile_) hipEventRecord(ln->anchor, resident ? ln->compute : ln->copy);
    if (ok && cur < segs.size() && !resident && !direct) ok = upload(cur, slot);
    while (ok && cur < segs.size() && !q.aborted()) {
      // (resident data: the next segment is taken when this one is done, so
      // two drivers take them in order)
      const size_t nxt = resident ? segs.size() : pipe.next_segment();
      // the next segment's upload goes behind this one's on the copy stream;
      // its ring slot was last read by the segment before this one, whose
      // kernels have completed (run_segment returns after its D2H)
      if (nxt < segs.size() && !resident && !(ok = upload(nxt, slot ^ 1))) break;
      const void* d_data = resident ? segs[cur].in.d_data : ln->ring[slot];
      StageIn stage;                     // (direct batches: this segment's prologue copies)
      if (direct) {
        // one small pinned batch: the segment prologue copies it (StageIn)
        const Segment& sg = segs[cur];
        std::memcpy(ln->h_off_pin[slot], sg.in.offsets, (sg.in.nfiles + 1) * sizeof(uint64_t));
        void* off_dev = nullptr;
        if (hipHostGetDevicePointer(&off_dev, ln->h_off_pin[slot], 0) != hipSuccess || !off_dev) {
          ok = false;
          e = "pinned offsets staging has no device view";
          break;
        }
        stage.src = h_dev + sg.b0;
        stage.dst = ln->ring[slot];
        stage.bytes = sg.bytes;
        stage.off_src = static_cast<const uint8_t*>(off_dev);
        stage.off_dst = reinterpret_cast<uint8_t*>(ln->off_slot[slot]);
        stage.off_bytes = (sg.in.nfiles + 1) * sizeof(uint64_t);
      } else if (!resident) {
        std::string* err = &e;
        auto wait_up = [&]() -> bool {
          HIP_OK(hipStreamWaitEvent(ln->compute, ln->up_done[slot], 0));
          return true;
        };
        if (!(ok = wait_up())) break;
      }
      std::unique_ptr<Job> job(new Job());
      job->seg = cur;
      ScanStats sst;
      const double h_start = ms_since(t_feed0);
      ok = run_segment(*dt, *ln, segs[cur], d_data, resident ? nullptr : ln->off_slot[slot], &sst, &job->out, &e,
                       &plan_pending, chain_p, /*defer_copy=*/true, direct ? &stage : nullptr);
      if (!ok) break;
      plan_pending();                    // (a rerun path may not have called it)
      if (host_profile_) {
        // GPU timeline of this segment from the scan's anchor event
        float ub = 0, ud = 0, k1a = 0, k1b = 0, k2b = 0;
        if (!resident && !direct) {
          hipEventElapsedTime(&ub, ln->anchor, ln->up_begin[slot]);
          hipEventElapsedTime(&ud, ln->anchor, ln->up_done[slot]);
        }
        hipEventElapsedTime(&k1a, ln->anchor, ln->ev[0]);
        hipEventElapsedTime(&k1b, ln->anchor, ln->ev[1]);
        hipEventElapsedTime(&k2b, ln->anchor, ln->ev[3]);
        std::fprintf(stderr, "[tsg tl] seg %zu: host %.3f-%.3f ms; gpu upload %.3f-%.3f, K1 %.3f-%.3f, K2 done %.3f\n",
                     cur, h_start, ms_since(t_feed0), ub, ud, k1a, k1b, k2b);
      }
      if (!resident && !direct) {
        float h2d = 0;
        if (hipEventElapsedTime(&h2d, ln->up_begin[slot], ln->up_done[slot]) == hipSuccess) sst.h2d_ms += h2d;
        const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t_feed0).count();
        int64_t prev = feed_end_ns.load();
        while (ns > prev && !feed_end_ns.compare_exchange_weak(prev, ns)) {}
      }
      add_stats(&dst, sst);
      pending = std::move(job);
      cur = resident ? pipe.next_segment() : nxt;
      slot ^= 1;
    }
    if (ok) plan_pending();
    } catch (const std::exception& x) {
      ok = false;
      e = std::string("host exception in the device driver: ") + x.what();
    } catch (...) {
      ok = false;
      e = "host exception in the device driver";
    }
    if (ln) {
      if (!ok) { hipStreamSynchronize(ln->copy); hipStreamSynchronize(ln->compute); }
      ln->pool_idle = nullptr;                   // (the flag is this scan's)
      release_lane(*dt, ln);
    }
    {
      std::lock_guard<std::mutex> lk(st_mu);
      add_stats(st, dst);
      gpu_busy = dual ? std::max(gpu_busy, ms_since(tb)) : gpu_busy + ms_since(tb);
    }
    if (!ok) *e_out = e;
    return ok;
  };
  CallCtx* cc = acquire_call();
  uint64_t nconf = 0, nfind = 0;
  double host_ms = 0;
  // one segment on one device (per-file Scan batches, small batches): the
  // driver runs on this thread -- a thread start and hand-off cost more than
  // the segment's GPU passes
  const bool inline_driver = segs.size() == 1 && drivers.size() == 1;
  std::string run_err;
  const bool run_ok = pipe.run(
      inline_driver, driver,
      [&] {
        // per-file result slots (hundreds of thousands for image layers) are set up
        // while the first segment's upload and GPU passes run
        results->clear();
        results->resize(in.nfiles);
        if (host_profile_) std::fprintf(stderr, "[tsg tl] %u result slots ready at %.3f ms\n", in.nfiles, ms_since(t_feed0));
      },
      [&](Job& job, int left) {
        auto th = std::chrono::steady_clock::now();
        const Segment& sg = segs[job.seg];
        const double c_start = host_profile_ ? ms_since(t_feed0) : 0.0;
        confirmer_idle.store(false, std::memory_order_release);
        // (drivers that block on an event leave every core to the pool)
        confirm_segment(*cc, sg, job.out, results->data() + sg.f0, &nconf, &nfind, left > 0 && !dual);
        confirmer_idle.store(true, std::memory_order_release);
        host_ms += ms_since(th);
        if (host_profile_) std::fprintf(stderr, "[tsg tl] seg %zu confirm %.3f-%.3f ms\n", job.seg, c_start, ms_since(t_feed0));
      },
      pop_spin_us_, &run_err);
  release_call(cc);
  if (!run_ok) { *err = run_err; return false; }
  st->bytes = total;
  st->files = in.nfiles;
  st->pieces = static_cast<uint32_t>(segs.size());
  st->devices = static_cast<uint32_t>(drivers.size());
  st->gpu_wall_ms = gpu_busy;
  st->host_ms = host_ms;
  st->confirm_files = nconf;
  st->findings = nfind;
  st->feed_ms = resident ? 0.0 : feed_end_ns.load() / 1e6;
  st->total_ms = ms_since(t0);
  return true;
}

}  // namespace tsg

extern "C" int tsg_alloc_pinned(size_t bytes, void** out) {
  if (!out) return -1;
  return hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? 0 : -4;
}

extern "C" void tsg_free_pinned(void* p) {
  if (p) hipHostFree(p);
}
