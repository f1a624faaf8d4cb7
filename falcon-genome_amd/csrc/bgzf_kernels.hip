// BGZF member inflation on gfx950 (the BAM reader in
// front of the PairHMM path; `fcs-genome htc` inflates every BAM block of its
// window before it can build a region).
//
// One 64-lane wave per member, many members per CU.  DEFLATE decoding is a
// serial chain (each symbol's bit position depends on the previous symbol), so
// the kernel's rate is set by how many members are in flight at once and by
// the latency of one symbol step:
// - the decode state is wave-uniform and kept in scalar registers (every
//   value the chain reads goes through readfirstlane), so the symbol step is
//   SALU work plus one LDS table read, with scalar branches;
// - a member holds only its Huffman tables in LDS (5.6 KiB, 54 VGPRs: 7
//   members per SIMD): the compressed payload is read from global memory 8 bytes
//   at a time, the output is written straight to its place in global memory
//   and back-references read it back past the vector L1 (agent-scope loads:
//   the bytes were written by this wave moments before);
// - match copies are split over the wave's lanes (byte k of a match is source
//   byte k mod distance, so overlapping copies need no serial loop);
// - the CRC-32 is computed over 64 lane chunks of the output and recombined
//   with the polynomial shift (bgzf_inflate.h).
// Per member the kernel moves its compressed bytes in and ≤ 64 KiB out (plus
// the CRC pass's re-read from L2); a batch is latency-bound, not HBM-bound.
#include <hip/hip_runtime.h>

#include "bgzf_inflate.h"
#include "fcship_internal.h"

namespace fcs {
namespace {

constexpr int kBgzfMax = 65536;  // a member's payload and output limit (BGZF)

__device__ __forceinline__ uint32_t rfl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

struct WaveLanes {
  __device__ static int id() { return (int)threadIdx.x; }
  __device__ static constexpr int n() { return 64; }
  template <class T>
  __device__ static T uni(T v) {
    return (T)rfl((uint32_t)v);
  }
  __device__ static uint32_t lane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
  // 8 bytes at p (global, any alignment; 8 more bytes readable): two aligned
  // 8-byte reads and a funnel shift, all uniform
  __device__ static uint64_t load64(const uint8_t* p) {
    const int mis = (int)((uintptr_t)p & 7);
    const uint64_t* a = reinterpret_cast<const uint64_t*>(p - mis);
    const uint64_t lo = a[0], hi = a[1];
    const int sh = 8 * mis;
    const uint64_t v = (lo >> sh) | ((hi << 1) << (63 - sh));
    return (uint64_t)rfl((uint32_t)v) | (uint64_t)rfl((uint32_t)(v >> 32)) << 32;
  }
  // every lane stores the same byte to the same address: one write, and no
  // exec-mask switch around it
  __device__ static void put(uint8_t* out, uint32_t pos, uint8_t v) { out[pos] = v; }
  __device__ static void copy(uint8_t* out, uint32_t to, uint32_t from) {
    out[to] = __hip_atomic_load(out + from, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // one wave: its memory operations are performed in order, so the lanes only
  // need the compiler to keep its accesses on the right side of this point
  __device__ static void sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
};

struct MemberLds {
  InfTables t;
};

__device__ __forceinline__ uint32_t le32(const uint8_t* p) {
  return rfl((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(64) void bgzf_inflate_kernel(const uint8_t* __restrict__ comp,
                                                          const int64_t* __restrict__ coff,
                                                          const int64_t* __restrict__ uoff, int32_t n,
                                                          uint8_t* __restrict__ out, int32_t* __restrict__ status) {
  __shared__ MemberLds S;
  const int m = (int)blockIdx.x, lane = (int)threadIdx.x;
  if (m >= n) return;
  const int64_t c0 = coff[m], clen = coff[m + 1] - c0, u0 = uoff[m], ulen = uoff[m + 1] - u0;
  const uint8_t* mem = comp + c0;
  if (clen < 20) {  // shorter than a gzip header and trailer: read nothing of it
    if (lane == 0) status[m] = FCS_BGZF_CORRUPT;
    return;
  }
  const int xlen = (int)rfl((uint32_t)mem[10] | (uint32_t)mem[11] << 8);
  const int64_t plen = clen - 12 - xlen - 8;
  if (plen < 0 || plen > kBgzfMax || ulen < 0 || ulen > kBgzfMax) {
    if (lane == 0) status[m] = FCS_BGZF_CORRUPT;
    return;
  }
  uint8_t* dst = out + u0;
  __syncthreads();
  uint32_t got = 0;
  int rc = inflate_raw<WaveLanes>(mem + 12 + xlen, (uint32_t)plen, dst, (uint32_t)ulen, &got, S.t);
  const uint32_t want_crc = le32(mem + clen - 8), isize = le32(mem + clen - 4);
  if (rc == kInfOk && ((int64_t)got != ulen || (int64_t)isize != ulen)) rc = kInfCorrupt;
  // CRC-32 of the output: contiguous lane chunks read back past the L1, each
  // shifted past the bytes after it
  const int ng = (int)got, chunk = (ng + 63) / 64;
  const int b = min(ng, lane * chunk), e = min(ng, b + chunk);
  // bitwise (no table: its 1 KiB of LDS would cost members in flight, and this
  // pass is ≈ 2% of a member's time)
  uint32_t c = 0xFFFFFFFFu;
  for (int q = b; q < e; ++q) {
    c ^= __hip_atomic_load(dst + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (kCrcPoly & (0u - (c & 1u)));
  }
  uint32_t part = e > b ? crc_shift(~c, (uint64_t)(ng - e)) : 0u;
  for (int off = 32; off > 0; off >>= 1) part ^= (uint32_t)__shfl_xor((int)part, off, 64);
  if (rc == kInfOk && part != want_crc) rc = FCS_BGZF_CRC;
  if (lane == 0) status[m] = rc;
}

static_assert(kInfOk == FCS_BGZF_OK && kInfCorrupt == FCS_BGZF_CORRUPT && kInfOverflow == FCS_BGZF_OVERFLOW,
              "decoder status codes are the C-ABI's");

}  // namespace

int launch_bgzf_inflate(const uint8_t* comp, const int64_t* coff, const int64_t* uoff, int32_t n, uint8_t* out,
                        int32_t* status, hipStream_t s) {
  if (n <= 0) return FCS_OK;
  hipLaunchKernelGGL(bgzf_inflate_kernel, dim3((unsigned)n), dim3(64), 0, s, comp, coff, uoff, n, out, status);
  FCS_HIP_CHECK(hipGetLastError());
  return FCS_OK;
}

}  // namespace fcs
