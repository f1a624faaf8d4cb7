// Raw DEFLATE decoding (RFC 1951) of one BGZF member's payload, written once
// for the device and the host: the device kernel (bgzf_kernels.hip) runs it on
// one wave per member with the member's input, output and Huffman tables in
// LDS; the host unit test (tools/micro/inflate_test.cpp) runs the very same
// code against zlib.  SURVEY.md §8 row f3 (the BAM/BGZF reader either side of
// the PairHMM path): `fcs-genome htc` spends most of its host decode time
// inflating BAM blocks.
//
// Decoding: a 64-bit LSB-first bit buffer refilled 7 bytes at a time;
// Huffman codes through a 2^10-entry table indexed by the next 10 stream bits
// (entry = length << 9 | symbol), longer codes by the canonical count / first
// walk (one bit at a time, as zlib's puff); stored, fixed and dynamic blocks.
// Every read is bounded by the input and every write by the output's
// capacity: a corrupt stream returns an error, never reads or writes outside
// its buffers.
//
// The policy `L` says who does what: `L::id` / `L::n` (the lanes that share a
// member: 1 on the host, the wave's 64 on the device), `L::load64(p)` (8 input
// bytes, little-endian, from p with p + 8 <= end and 8 more readable),
// `L::put(out, pos, byte)` (one lane writes a literal), `L::copy(out, to,
// from)` (a lane copies one byte written earlier: back-references), `L::uni(v)` (a value every
// lane holds alike: the device keeps the decode state in scalar registers),
// `L::lane(v, l)` (lane l's value of v; device only)
// and `L::sync()` (the lanes' writes visible to each other).  Every lane
// decodes the same symbols; the lanes split the table fills and the match
// copies.
#pragma once

#include <cstddef>
#include <cstdint>

namespace fcs {

constexpr int kInfFastBits = 10;

struct InfHuff {
  uint16_t fast[1 << kInfFastBits];  // len << 9 | sym (| 0x8000 for a literal in the lit table), 0: longer code
  uint16_t count[16];                // codes per length
  uint16_t sorted[288];              // symbols ordered by (length, symbol)
};

// The two tables one member needs at a time (the code-length code borrows
// dist) and the code lengths they are built from (LDS on the device).
struct InfTables {
  InfHuff lit, dist;
  uint8_t lens[320];
  uint8_t cl[20];
};

enum : int { kInfOk = 0, kInfCorrupt = 1, kInfOverflow = 2 };

// Offsets are 32-bit (a member is at most 64 KiB in and out), so the device
// keeps them in scalar registers with 32-bit compares.  A read past the input
// leaves `cnt` negative (checked at block ends): zero bits decode to some
// symbols, but every symbol either advances the output or ends the block, so a
// corrupt stream still ends (overflow or a negative count).
template <class L>
struct InfBits {
  const uint8_t* in;
  uint32_t at, n;
  uint64_t buf;
  int cnt;
  __host__ __device__ __forceinline__ void refill() {
    if (n - at >= 8) {
      // 7 or 8 whole bytes: the buffer ends up holding 56..63 bits
      buf |= L::load64(in + at) << cnt;  // uniform (L::load64 says so)
      at += (uint32_t)(63 - cnt) >> 3;
      cnt |= 56;
      return;
    }
    if (cnt < 0) return;
    while (cnt <= 56 && at < n) {
      buf |= (uint64_t)L::uni(in[at++]) << cnt;
      cnt += 8;
    }
  }
  __host__ __device__ __forceinline__ uint32_t peek(int k) {
    if (cnt < k) refill();
    return (uint32_t)(buf & ((1ull << k) - 1));
  }
  __host__ __device__ __forceinline__ void drop(int k) {
    buf >>= k;
    cnt -= k;
  }
  __host__ __device__ __forceinline__ uint32_t get(int k) {
    if (k == 0) return 0;
    const uint32_t v = peek(k);
    drop(k);
    return v;
  }
  __host__ __device__ __forceinline__ bool over() const { return cnt < 0; }
};

// Canonical Huffman table from code lengths (len[0..n)); false when the
// lengths over-subscribe the code space.  Counts and the sorted symbol list
// are built by every lane alike; the fast table's entries are split.
template <class L, bool kLitFlag = false>
__host__ __device__ inline bool inf_build(InfHuff& h, const uint8_t* len, int n) {
  // per-length code counts: on the device lane l holds the count of length l
  // in one register (read back with L::lane), on the host an array
  uint32_t mine = 0, cnt_host[16];
  if constexpr (L::n() > 1) {
#pragma unroll 1
    for (int s = 0; s < n; ++s) mine += (uint32_t)(L::uni(len[s]) == L::id());
  } else {
    for (int l = 0; l < 16; ++l) cnt_host[l] = 0;
    for (int s = 0; s < n; ++s) cnt_host[len[s]]++;
  }
  uint32_t cnt[16];
#pragma unroll
  for (int l = 0; l < 16; ++l) {
    if constexpr (L::n() > 1) cnt[l] = l ? L::lane(mine, l) : 0;
    else cnt[l] = l ? cnt_host[l] : 0;
  }
  int left = 1;
#pragma unroll
  for (int l = 1; l < 16; ++l) {
    left <<= 1;
    left -= (int)cnt[l];
    if (left < 0) return false;
  }
  uint32_t o = 0, my_off = 0;
#pragma unroll
  for (int l = 0; l < 16; ++l) {
    if (L::id() == 0) h.count[l] = (uint16_t)cnt[l];
    if (l == L::id()) my_off = o;  // the device lane of length l
    o += cnt[l];
  }
  // symbols in (length, symbol) order: on the device lane l (1..15) places
  // the length-l ones; the host's single lane all of them
  if constexpr (L::n() > 1) {
#pragma unroll 1  // unrolled, the symbol numbers became 29 hoisted VGPR constants
    for (int s = 0; s < n; ++s) {
      const int l = L::uni(len[s]);
      if (l && l == L::id()) h.sorted[my_off++] = (uint16_t)s;
    }
  } else {
    uint32_t at[16];
    at[0] = at[1] = 0;
    for (int l = 2; l < 16; ++l) at[l] = at[l - 1] + cnt[l - 1];
    for (int s = 0; s < n; ++s)
      if (len[s]) h.sorted[at[len[s]]++] = (uint16_t)s;
  }
  // fast entries: entry i holds the code that the bit-reversed 10-bit index
  // starts with (canonical codes walked per length, as the slow decode does)
  L::sync();
  for (int i = L::id(); i < (1 << kInfFastBits); i += L::n()) {
    int r = 0;
    for (int b = 0; b < kInfFastBits; ++b) r |= ((i >> b) & 1) << (kInfFastBits - 1 - b);
    int first = 0, index = 0;
    uint16_t e = 0;
    for (int l = 1; l <= kInfFastBits; ++l) {
      const int code = r >> (kInfFastBits - l);
      const int c = (int)cnt[l];
      if (code - first < c) {
        const int sym = h.sorted[index + code - first];
        // the literal/length table marks literals (bit 15): the literal-run
        // loop's exit test is one bit and the output room
        e = (uint16_t)(l << 9 | sym | (kLitFlag && sym < 256 ? 0x8000 : 0));
        break;
      }
      index += c;
      first = (first + c) << 1;
    }
    h.fast[i] = e;
  }
  L::sync();
  return true;
}

// One symbol; kInfBadSym (above every valid literal/length and distance
// symbol, so the callers' range checks catch it) on an invalid code.
constexpr int kInfBadSym = 0x7FFF;

// Codes longer than the fast table, bit by bit (rare: kept rolled).
template <class L>
__host__ __device__ inline int inf_decode_slow(InfBits<L>& b, const InfHuff& h) {
  int code = 0, first = 0, index = 0;
#pragma unroll 1
  for (int l = 1; l < 16; ++l) {
    code |= (int)b.get(1);
    const int count = L::uni(h.count[l]);
    if (code - count < first) return L::uni(h.sorted[index + (code - first)]);
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return kInfBadSym;
}

template <class L>
__host__ __device__ __forceinline__ int inf_decode(InfBits<L>& b, const InfHuff& h) {
  const uint32_t e = L::uni(h.fast[b.peek(kInfFastBits)]);
  if (e) {
    b.drop((int)(e >> 9));
    return (int)(e & 511u);
  }
  return inf_decode_slow(b, h);
}

__host__ __device__ __forceinline__ void inf_len_base(int i, int& base, int& extra) {
  if (i < 8) base = 3 + i, extra = 0;
  else if (i == 28) base = 258, extra = 0;
  else extra = (i - 4) >> 2, base = ((4 + (i & 3)) << extra) + 3;
}
__host__ __device__ __forceinline__ void inf_dist_base(int i, int& base, int& extra) {
  if (i < 4) base = 1 + i, extra = 0;
  else extra = (i - 2) >> 1, base = ((2 + (i & 1)) << extra) + 1;
}

// The literal/length and distance codes of one block up to its end-of-block
// symbol.  One refill per symbol: a refill leaves 56+ bits unless the input is
// nearly used up, and a literal/length code (15), its extra bits (5), a
// distance code (15) and its extra bits (13) take at most 48.
template <class L>
__host__ __device__ __forceinline__ int inf_codes(InfBits<L>& b, const InfTables& t, uint8_t* out, uint32_t cap,
                                                  uint32_t& pos) {
  for (;;) {
    if (b.cnt < 48) b.refill();
    // literal runs in a loop of their own with one combined exit test (a
    // literal from the fast table and room for it): its step is a table read,
    // a shift, a store and a refill test, with no per-exit flow flags
    uint32_t e = L::uni(t.lit.fast[(uint32_t)b.buf & ((1u << kInfFastBits) - 1)]);
    while ((e >> 15) && pos < cap) {
      b.drop((int)((e >> 9) & 15u));
      L::put(out, pos++, (uint8_t)e);
      if (b.cnt < kInfFastBits) b.refill();
      e = L::uni(t.lit.fast[(uint32_t)b.buf & ((1u << kInfFastBits) - 1)]);
    }
    if (b.cnt < 48) b.refill();
    int sym;
    {
      if (e) {
        b.drop((int)((e >> 9) & 15u));
        sym = (int)(e & 511u);
      } else {
        sym = inf_decode_slow(b, t.lit);
      }
    }
    if (sym < 256) {
      if (pos >= cap) return kInfOverflow;
      L::put(out, pos++, (uint8_t)sym);
      continue;
    }
    if (sym == 256) return b.over() ? kInfCorrupt : kInfOk;
    if (sym > 285) return kInfCorrupt;
    int lbase, lextra, dbase, dextra;
    inf_len_base(sym - 257, lbase, lextra);
    const int len = lbase + (int)((uint32_t)b.buf & ((1u << lextra) - 1));
    b.drop(lextra);
    int dsym;
    {
      const uint32_t e = L::uni(t.dist.fast[(uint32_t)b.buf & ((1u << kInfFastBits) - 1)]);
      if (e) {
        b.drop((int)(e >> 9));
        dsym = (int)(e & 511u);
      } else {
        dsym = inf_decode_slow(b, t.dist);
      }
    }
    if (dsym > 29) return kInfCorrupt;
    inf_dist_base(dsym, dbase, dextra);
    const uint32_t dist = (uint32_t)dbase + ((uint32_t)b.buf & ((1u << dextra) - 1));
    b.drop(dextra);
    if (dist > pos) return kInfCorrupt;
    if ((uint32_t)len > cap - pos) return kInfOverflow;
    // the match repeats the last `dist` bytes: byte k of it is source byte
    // k mod dist (overlapping copies, as DEFLATE means)
    L::sync();
    const uint32_t src = pos - dist;
    const int d = (int)dist;
    if (d >= len) {  // no overlap: a straight copy (the modulo below is ≈ 20 VALU ops)
      for (int k = L::id(); k < len; k += L::n()) L::copy(out, pos + k, src + k);
    } else {
      for (int k = L::id(); k < len; k += L::n()) L::copy(out, pos + k, src + (uint32_t)(k % d));
    }
    L::sync();
    pos += (uint32_t)len;
  }
}

// Raw DEFLATE in[0, n) -> out[0, cap); *produced = bytes written.
template <class L>
__host__ __device__ inline int inflate_raw(const uint8_t* in, uint32_t n, uint8_t* out, uint32_t cap,
                                           uint32_t* produced, InfTables& t) {
  InfBits<L> b{in, 0, n, 0, 0};
  uint32_t pos = 0;
  int rc = kInfOk;
  for (;;) {
    const uint32_t bfinal = b.get(1), btype = b.get(2);
    if (btype == 0) {  // stored: to a byte boundary, LEN, NLEN, LEN raw bytes
      if (b.over()) { rc = kInfCorrupt; break; }
      b.drop(b.cnt & 7);
      const uint32_t len = b.get(16), nlen = b.get(16);
      if ((len ^ 0xFFFFu) != nlen || b.over()) { rc = kInfCorrupt; break; }
      if (len > cap - pos) { rc = kInfOverflow; break; }
      // whole bytes still in the bit buffer, then the rest straight from the
      // input, split over the lanes
      uint32_t k = 0;
      for (; k < len && b.cnt >= 8; ++k) L::put(out, pos + k, (uint8_t)b.get(8));
      const uint32_t rest = len - k;
      if (rest > b.n - b.at) { rc = kInfCorrupt; break; }
      L::sync();
      for (uint32_t j = (uint32_t)L::id(); j < rest; j += (uint32_t)L::n()) out[pos + k + j] = b.in[b.at + j];
      L::sync();
      b.at += rest;
      if (rest) b.buf = 0, b.cnt = 0;
      pos += len;
    } else if (btype == 1 || btype == 2) {
      uint8_t* const lens = t.lens;
      int nlit = 288, ndist = 30;
      if (btype == 1) {
        for (int s = L::id(); s < 320; s += L::n()) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
        L::sync();
      } else {
        nlit = (int)b.get(5) + 257;
        ndist = (int)b.get(5) + 1;
        const int ncode = (int)b.get(4) + 4;
        if (nlit > 286 || ndist > 30) { rc = kInfCorrupt; break; }
        // code-length code lengths in the order 16 17 18 0 8 7 9 6 10 5 11 4 12 3 13 2 14 1 15
        uint8_t* const cl = t.cl;
        if (L::id() == 0)
          for (int s = 0; s < 19; ++s) cl[s] = 0;
        L::sync();
        for (int s = 0; s < ncode; ++s) {
          const uint8_t v = (uint8_t)b.get(3);
          const int slot = s < 3 ? 16 + s : s == 3 ? 0 : (s & 1) ? 8 - (s - 3) / 2 : 8 + (s - 4) / 2;
          if (L::id() == 0) cl[slot] = v;
        }
        L::sync();
        if (!inf_build<L>(t.dist, cl, 19)) { rc = kInfCorrupt; break; }
        int s = 0;
        while (s < nlit + ndist) {
          const int sym = inf_decode(b, t.dist);
          if (sym > 18) { rc = kInfCorrupt; break; }
          if (sym < 16) {
            if (L::id() == 0) lens[s] = (uint8_t)sym;
            ++s;
            continue;
          }
          int rep, val = 0;
          if (sym == 16) {
            if (s == 0) { rc = kInfCorrupt; break; }
            L::sync();
            val = L::uni(lens[s - 1]);
            rep = 3 + (int)b.get(2);
          } else if (sym == 17) {
            rep = 3 + (int)b.get(3);
          } else {
            rep = 11 + (int)b.get(7);
          }
          if (s + rep > nlit + ndist) { rc = kInfCorrupt; break; }
          for (int k = L::id(); k < rep; k += L::n()) lens[s + k] = (uint8_t)val;
          s += rep;
        }
        if (rc != kInfOk) break;
        L::sync();
        if (L::uni(lens[256]) == 0) { rc = kInfCorrupt; break; }  // no end-of-block code
        // the distance lengths follow the literal / length ones: moved up to
        // 288 (the ranges overlap when nlit + ndist > 288: the device reads
        // them into lane registers first, the host copies backwards), the
        // unused entries of both codes zeroed
        if constexpr (L::n() > 1) {
          const int k = L::id();
          const uint8_t v = k < ndist ? lens[nlit + k] : 0;
          L::sync();
          if (k < 30) lens[288 + k] = v;
        } else {
          for (int k = ndist - 1; k >= 0; --k) lens[288 + k] = lens[nlit + k];
          for (int k = ndist; k < 30; ++k) lens[288 + k] = 0;
        }
        L::sync();
        for (int k = nlit + L::id(); k < 288; k += L::n()) lens[k] = 0;
        L::sync();
      }
      if (!inf_build<L, true>(t.lit, lens, 288) || !inf_build<L>(t.dist, lens + 288, 30)) { rc = kInfCorrupt; break; }
      if ((rc = inf_codes<L>(b, t, out, cap, pos)) != kInfOk) break;
    } else {
      rc = kInfCorrupt;
      break;
    }
    if (b.over()) { rc = kInfCorrupt; break; }
    if (bfinal) break;
  }
  L::sync();
  *produced = pos;
  return rc;
}

// CRC-32 (IEEE, reflected 0xEDB88320).  The device splits a member's output
// over its lanes: crc(A || B) = shift(crc(A), |B|) ^ crc(B), the shift being
// a multiplication by x^(8 |B|) modulo the polynomial (bit 31 = x^0 in the
// reflected form).
constexpr uint32_t kCrcPoly = 0xEDB88320u;

__host__ __device__ inline uint32_t crc32_entry(uint32_t i) {
  uint32_t c = i;
  for (int k = 0; k < 8; ++k) c = (c & 1) ? kCrcPoly ^ (c >> 1) : c >> 1;
  return c;
}

// a * b modulo the CRC polynomial (reflected operands)
__host__ __device__ inline uint32_t crc_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int k = 31; k >= 0; --k) {
    if ((a >> k) & 1) p ^= b;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

// x^(8 n) modulo the polynomial: squares of x^8 for the set bits of n
__host__ __device__ inline uint32_t crc_x8n(uint64_t n) {
  uint32_t p = 1u << 31, sq = 1u << 23;  // x^0, x^8
  while (n) {
    if (n & 1) p = crc_mulmod(sq, p);
    sq = crc_mulmod(sq, sq);
    n >>= 1;
  }
  return p;
}

__host__ __device__ inline uint32_t crc_shift(uint32_t crc, uint64_t nbytes) {
  return crc_mulmod(crc_x8n(nbytes), crc);
}

}  // namespace fcs
