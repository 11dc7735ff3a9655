// GPU-side CR strip: the secret analyzer's
//   content = bytes.ReplaceAll(content, []byte("\r"), []byte(""))
// (pkg/fanal/analyzer/secret/secret.go:121) for every text file of a packed
// device batch.  Removing bytes never moves one across a file boundary, so
// the batch's stripped image is one stream compaction of the whole batch;
// each file's new start is the output position of its first input byte.
//
// One pass (decoupled look-back, as in single-pass prefix scans): each
// workgroup takes the next 32 KiB tile from a counter; each of its 8 waves
// holds 4 KiB in registers (lane l: bytes [16l, 16l + 16) of each 1 KiB
// sub-tile).  The workgroup publishes its kept-byte count, then reads the
// status words of the 512 preceding tiles at once (one per thread) back to the
// nearest published inclusive prefix, publishes its own inclusive prefix and
// writes the kept bytes and the new start of every file that begins in it.
// HBM traffic N + N' (read once, write once) plus 8 bytes of status per tile;
// a small kernel first finds the first file of each 4 KiB wave tile.  With a
// 512-tile window the prefix frontier moves 16 MB per L2 round trip, well
// ahead of HBM (a one-wave, one-status-at-a-time look-back measured 1.9 s for
// 10 GB: the frontier then moved one tile per round trip).
// Output goes to HBM as aligned dwords through a per-wave LDS staging line
// (byte stores only at the two partial dwords at a sub-tile's ends, which the
// neighbouring sub-tiles complete); a sub-tile with no '\r' whose output is
// 16-byte aligned (every one before the batch's first '\r') is stored directly.
#include "crstrip.h"

#include <cstdlib>

namespace tsg {
namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr uint32_t kCrSub = 1024;            // bytes per wave step (64 lanes x 16 B)
constexpr uint32_t kCrWaves = 8;             // waves per workgroup
constexpr uint32_t kCrThreads = 64 * kCrWaves;          // = the look-back window (tiles)
// tile status word: state in the top two bits, kept-byte count below
constexpr unsigned long long kCrAggregate = 1ull << 62, kCrInclusive = 2ull << 62, kCrValue = (1ull << 62) - 1;

// bit k (k < 4): byte k of d is '\r'
__device__ __forceinline__ uint32_t cr_bits(uint32_t d) {
  const uint32_t x = d ^ 0x0d0d0d0du;
  const uint32_t z = ~((((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x)) & 0x80808080u;   // bit 7 of a byte: byte == '\r'
  return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

__device__ __forceinline__ uint32_t cr_mask16(v4u w) {
  return cr_bits(w.x) | (cr_bits(w.y) << 4) | (cr_bits(w.z) << 8) | (cr_bits(w.w) << 12);
}

// 16 bytes at p; *valid = mask of the bytes below `total` (the batch end need
// not be 16-byte aligned, and nothing past it is read)
__device__ __forceinline__ v4u cr_load(const uint8_t* __restrict__ src, uint64_t p, uint64_t total, uint32_t* valid) {
  if (p + 16 <= total) {
    *valid = 0xffffu;
    return __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src + p));
  }
  uint32_t b[4] = {0, 0, 0, 0}, v = 0;
  for (uint32_t k = 0; k < 16 && p + k < total; ++k) {
    b[k >> 2] |= static_cast<uint32_t>(src[p + k]) << ((k & 3) * 8);
    v |= 1u << k;
  }
  *valid = v;
  return v4u{b[0], b[1], b[2], b[3]};
}

// first[t] = the first file whose start is >= t * wave_tile (lower_bound)
__global__ __launch_bounds__(256) void tsg_cr_tile_first(const uint64_t* __restrict__ offsets, uint32_t nfiles,
                                                         uint32_t ntiles, uint32_t wave_tile,
                                                         uint32_t* __restrict__ first) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const uint64_t x = static_cast<uint64_t>(t) * wave_tile;
  uint32_t lo = 0, hi = nfiles + 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (offsets[mid] < x) lo = mid + 1; else hi = mid;
  }
  first[t] = lo;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t u = __shfl_up(v, d);
    if (lane >= d) v += u;
  }
  return v;
}

// status[t] of every tile and status[ntiles] (the tile counter) start at 0.
template <uint32_t kCrSubs, int kMinWaves>
__global__ __launch_bounds__(kCrThreads, kMinWaves) void tsg_cr_strip(const uint8_t* __restrict__ src, uint64_t total,
                                                           uint32_t ntiles, uint32_t nwt,
                                                           const uint32_t* __restrict__ first,
                                                           const uint64_t* __restrict__ offsets, uint32_t nfiles,
                                                           uint8_t* __restrict__ dst, uint64_t* __restrict__ new_off,
                                                           unsigned long long* __restrict__ status,
                                                           uint64_t* __restrict__ out_total,
                                                           unsigned long long* __restrict__ dbg) {
  constexpr uint32_t kCrWaveTile = kCrSub * kCrSubs;     // bytes per wave
  __shared__ __attribute__((aligned(16))) uint8_t stage[kCrWaves][kCrSub + 16];
  __shared__ uint32_t s_tile, s_wt[kCrWaves], s_agg[kCrWaves], s_inc, s_nr;
  __shared__ unsigned long long s_incval;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint8_t* lb = stage[wv];
  if (threadIdx.x == 0) s_tile = atomicAdd(reinterpret_cast<unsigned int*>(status + ntiles), 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  if (tile >= ntiles) return;                // the whole workgroup
  const uint32_t wt = tile * kCrWaves + wv;  // this wave's 4 KiB tile
  const uint64_t t0 = static_cast<uint64_t>(wt) * kCrWaveTile;
  v4u w[kCrSubs];
  uint32_t keep[kCrSubs];
#pragma unroll
  for (uint32_t j = 0; j < kCrSubs; ++j) {
    uint32_t valid;
    w[j] = cr_load(src, t0 + j * kCrSub + lane * 16u, total, &valid);
    keep[j] = valid;
  }
  uint32_t k[kCrSubs], excl[kCrSubs], K[kCrSubs], T = 0;
#pragma unroll
  for (uint32_t j = 0; j < kCrSubs; ++j) {
    keep[j] &= ~cr_mask16(w[j]);
    k[j] = __popc(keep[j]);
    const uint32_t incl = wave_incl_scan(k[j], lane);
    excl[j] = incl - k[j];
    K[j] = __shfl(incl, 63);
    T += K[j];
  }
  if (lane == 0) s_wt[wv] = T;
  __syncthreads();
  uint32_t wbase = 0, TT = 0;                // kept bytes of the earlier waves / of the tile
#pragma unroll
  for (uint32_t i = 0; i < kCrWaves; ++i) {
    if (i < wv) wbase += s_wt[i];
    TT += s_wt[i];
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(status + tile, (tile == 0 ? kCrInclusive : kCrAggregate) | TT, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // look-back: thread i reads the status of tile p - i; every earlier tile is
  // held by a running or finished workgroup, and tile 0 publishes at once.
  // Status words are relaxed device-scope atomics: they carry the counts
  // themselves and order nothing else (release / acquire at device scope
  // write back / invalidate the XCD's L2 on every access: measured 64 ms
  // instead of a few for 10 GB)
  unsigned long long before = 0;
  for (long long p = static_cast<long long>(tile) - 1; p >= 0;) {
    const uint32_t i = threadIdx.x;
    const unsigned long long v = static_cast<long long>(i) <= p
        ? __hip_atomic_load(status + (p - i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
        : kCrAggregate;                      // past tile 0: never reached (tile 0 is inclusive)
    if (i == 0) { s_inc = 0xffffffffu; s_nr = 0xffffffffu; }
    __syncthreads();
    if (v & kCrInclusive) atomicMin(&s_inc, i);
    if (v == 0) atomicMin(&s_nr, i);
    __syncthreads();
    const uint32_t inc = s_inc, nr = s_nr;
    if (dbg && i == 0) atomicAdd(dbg + (nr < inc ? 0 : 1), 1ull);
    if (dbg && i == 0 && nr < inc) atomicAdd(dbg + 2, static_cast<unsigned long long>(nr));
    if (dbg && i == 0 && nr >= inc && inc != 0xffffffffu) atomicAdd(dbg + 3, static_cast<unsigned long long>(inc));
    if (nr < inc) {                          // a nearer tile has not published yet
      __syncthreads();
      __builtin_amdgcn_s_sleep(2);
      continue;
    }
    uint32_t x = i < inc ? static_cast<uint32_t>(v & kCrValue) : 0u;   // aggregates (<= 32 KiB each)
    if (i == inc) s_incval = v & kCrValue;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d);
    if (lane == 0) s_agg[wv] = x;
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < kCrWaves; ++q) before += s_agg[q];
    if (inc != 0xffffffffu) {
      before += s_incval;
      break;
    }
    __syncthreads();
    p -= kCrThreads;
  }
  if (threadIdx.x == 0 && tile > 0)
    __hip_atomic_store(status + tile, kCrInclusive | (before + TT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t out = before + wbase;
  uint32_t f = first[wt];
  uint64_t next_start = offsets[f];          // wave-uniform: the next file start at or after the sub-tile
#pragma unroll
  for (uint32_t j = 0; j < kCrSubs; ++j) {
    const uint64_t s0 = t0 + j * kCrSub;
    if (s0 >= total) break;
    const bool plain = __ballot(keep[j] != 0xffffu) == 0;   // full sub-tile without '\r'
    if (plain && (out & 15u) == 0) {
      __builtin_nontemporal_store(w[j], reinterpret_cast<v4u*>(dst + out + lane * 16u));
    } else if (K[j]) {
      const uint32_t q0 = static_cast<uint32_t>(out & 3u);   // stage byte q holds output byte (out & ~3) + q
      if (plain && q0 == 0) {
        *reinterpret_cast<v4u*>(lb + lane * 16u) = w[j];
      } else {
        const uint32_t ws[4] = {w[j].x, w[j].y, w[j].z, w[j].w};
        uint32_t q = q0 + excl[j];
#pragma unroll
        for (int b = 0; b < 16; ++b) {
          if ((keep[j] >> b) & 1u) {
            lb[q] = static_cast<uint8_t>(ws[b >> 2] >> ((b & 3) * 8));
            ++q;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const uint64_t a0 = out - q0, e = out + K[j];
      const uint32_t ndw = static_cast<uint32_t>((e - a0 + 3) >> 2);
      for (uint32_t d = lane; d < ndw; d += 64) {
        const uint64_t g = a0 + 4ull * d;
        const uint32_t v = *reinterpret_cast<const uint32_t*>(lb + 4 * d);
        if (g >= out && g + 4 <= e) {
          *reinterpret_cast<uint32_t*>(dst + g) = v;
        } else {
          for (uint32_t b = 0; b < 4; ++b)
            if (g + b >= out && g + b < e) dst[g + b] = static_cast<uint8_t>(v >> (8 * b));
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // files starting in this sub-tile: new start = output position of their first byte
    const uint64_t s1 = min(s0 + kCrSub, total);
    while (next_start < s1) {
      const uint32_t idx = f + lane;
      const uint64_t o = idx <= nfiles ? offsets[idx] : ~0ull;
      const bool in = o < s1;                // o >= s0: files are sorted and f is past the earlier ones
      const uint32_t wi = in ? static_cast<uint32_t>((o - s0) >> 4) : 0u;
      const uint32_t pe = __shfl(excl[j], wi), pk = __shfl(keep[j], wi);
      if (in) new_off[idx] = out + pe + __popc(pk & ((1u << (o & 15u)) - 1u));
      f += static_cast<uint32_t>(__popcll(__ballot(in)));
      next_start = f <= nfiles ? offsets[f] : ~0ull;
    }
    out += K[j];
  }
  if (wt == nwt - 1) {                       // files starting at the batch end, and the stripped total
    for (uint32_t i = f + lane; i <= nfiles; i += 64) new_off[i] = out;
    if (lane == 0) *out_total = out;
  }
}

}  // namespace

unsigned long long* dbg_ = nullptr;   // TSG_CR_DEBUG: look-back counters (measurement)
void cr_strip_dbg(unsigned long long* d) { dbg_ = d; }

// TSG_CR_VARIANT (measurement): sub-tiles per wave x minimum waves per SIMD
int cr_variant_ = 0;
struct CrVariant { uint32_t subs; const void* fn; };
CrVariant cr_variant() {
  switch (cr_variant_) {
    case 1: return {4, reinterpret_cast<const void*>(&tsg_cr_strip<4, 6>)};
    case 2: return {2, reinterpret_cast<const void*>(&tsg_cr_strip<2, 1>)};
    case 3: return {2, reinterpret_cast<const void*>(&tsg_cr_strip<2, 8>)};
    case 4: return {1, reinterpret_cast<const void*>(&tsg_cr_strip<1, 8>)};
    default: return {4, reinterpret_cast<const void*>(&tsg_cr_strip<4, 1>)};
  }
}

size_t cr_strip_scratch_bytes(uint64_t total) {
  const uint64_t wave_tile = kCrSub;             // the smallest variant's
  const uint64_t ntiles = (total + wave_tile * kCrWaves - 1) / (wave_tile * kCrWaves);
  const uint64_t nwt = (total + wave_tile - 1) / wave_tile;
  return 64 + (ntiles + 1) * 8 + nwt * 4 + 64;
}

bool cr_strip_launch(const uint8_t* src, const uint64_t* offsets, uint32_t nfiles, uint64_t total, uint8_t* dst,
                     uint64_t* new_off, void* scratch, hipStream_t s, std::string* err) {
  static const bool once = [] {
    if (const char* c = std::getenv("TSG_CR_VARIANT")) cr_variant_ = std::atoi(c);
    return true;
  }();
  (void)once;
  const CrVariant v = cr_variant();
  const uint64_t wave_tile = kCrSub * v.subs, tile = wave_tile * kCrWaves;
  const uint64_t nt64 = (total + tile - 1) / tile, nwt64 = (total + wave_tile - 1) / wave_tile;
  if (nwt64 >= 0xffffffffull) { *err = "batch too large for the CR strip"; return false; }
  const uint32_t ntiles = static_cast<uint32_t>(nt64), nwt = static_cast<uint32_t>(nwt64);
  uint8_t* sp = static_cast<uint8_t*>(scratch);
  uint64_t* d_total = reinterpret_cast<uint64_t*>(sp);
  unsigned long long* status = reinterpret_cast<unsigned long long*>(sp + 64);
  uint32_t* first = reinterpret_cast<uint32_t*>(sp + 64 + (nt64 + 1) * 8);
  if (ntiles == 0) {                         // every file is empty
    if (hipMemsetAsync(new_off, 0, (static_cast<size_t>(nfiles) + 1) * 8, s) != hipSuccess ||
        hipMemsetAsync(d_total, 0, 8, s) != hipSuccess) {
      *err = "CR strip: memset failed";
      return false;
    }
    return true;
  }
  if (hipMemsetAsync(status, 0, (nt64 + 1) * 8, s) != hipSuccess) { *err = "CR strip: memset failed"; return false; }
  hipLaunchKernelGGL(tsg_cr_tile_first, dim3((nwt + 255) / 256), dim3(256), 0, s, offsets, nfiles, nwt,
                     static_cast<uint32_t>(wave_tile), first);
  void* args[] = {&src, &total, const_cast<uint32_t*>(&ntiles), const_cast<uint32_t*>(&nwt), &first, &offsets, &nfiles,
                  &dst, &new_off, &status, &d_total, &dbg_};
  if (hipLaunchKernel(v.fn, dim3(ntiles), dim3(kCrThreads), args, 0, s) != hipSuccess) {
    *err = "CR strip launch failed";
    return false;
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) { *err = std::string("CR strip launch: ") + hipGetErrorString(e); return false; }
  return true;
}

}  // namespace tsg
