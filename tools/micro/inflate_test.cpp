// Host check of csrc/bgzf_inflate.h (the device kernel's DEFLATE decoder and
// CRC combination) against zlib: random / text / BAM-like / run-heavy
// payloads at every zlib level and strategy, plus flipped-bit and truncated
// streams (any status, never an out-of-bounds access: build with
// -fsanitize=address,undefined).
//   g++ -O2 -fsanitize=address,undefined -Ifalcon-genome_amd/csrc \
//       tools/micro/inflate_test.cpp -o /tmp/inflate_test -lz
#define __host__
#define __device__
#define __forceinline__ inline
#include "bgzf_inflate.h"

#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

using namespace fcs;

struct HostLanes {
  static int id() { return 0; }
  static constexpr int n() { return 1; }
  template <class T>
  static T uni(T v) { return v; }
  static void copy(uint8_t* out, uint32_t to, uint32_t from) { out[to] = out[from]; }
  static uint64_t load64(const uint8_t* p) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    return v;
  }
  static void put(uint8_t* out, uint32_t pos, uint8_t v) { out[pos] = v; }
  static void sync() {}
};

static std::vector<uint8_t> deflate_raw(const std::vector<uint8_t>& in, int level, int strategy) {
  z_stream zs{};
  deflateInit2(&zs, level, Z_DEFLATED, -15, 8, strategy);
  std::vector<uint8_t> out(compressBound(in.size()) + 64);
  zs.next_in = const_cast<Bytef*>(in.data());
  zs.avail_in = (uInt)in.size();
  zs.next_out = out.data();
  zs.avail_out = (uInt)out.size();
  if (deflate(&zs, Z_FINISH) != Z_STREAM_END) {
    std::puts("deflate failed");
    std::exit(2);
  }
  out.resize(zs.total_out);
  deflateEnd(&zs);
  return out;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
  std::mt19937 rng(7);
  InfTables* t = new InfTables;
  const char* line = "chr1\t100\t.\tA\t<NON_REF>\t.\t.\tEND=105\tGT:DP\t0/0:30\n";
  const size_t line_len = std::strlen(line);
  const int strategies[5] = {Z_DEFAULT_STRATEGY, Z_FIXED, Z_HUFFMAN_ONLY, Z_RLE, Z_FILTERED};
  int bad = 0, crc_bad = 0;
  for (int it = 0; it < iters; ++it) {
    size_t n = rng() % 65281;
    if (it % 10 == 0) n = rng() % 64;
    std::vector<uint8_t> d(n);
    const int kind = it % 5;
    for (size_t i = 0; i < n; ++i) {
      if (kind == 0) d[i] = (uint8_t)rng();
      else if (kind == 1) d[i] = (uint8_t)"ACGT\t0123456789\n"[rng() % 16];
      else if (kind == 2) d[i] = (i % 100 < 60) ? (uint8_t)line[i % line_len] : (uint8_t)(rng() % 32 + 33);
      else if (kind == 3) d[i] = (rng() % 10 == 0) ? (uint8_t)rng() : 'A';
      else d[i] = i < 8 ? (uint8_t)rng() : d[i - 1 - rng() % 8];
    }
    const int level = (int)(rng() % 10), strategy = strategies[rng() % 5];
    const std::vector<uint8_t> c = deflate_raw(d, level, strategy);
    std::vector<uint8_t> o(n + 16, 0xAA);
    uint32_t got = 0;
    const int rc = inflate_raw<HostLanes>(c.data(), (uint32_t)c.size(), o.data(), (uint32_t)n, &got, *t);
    if (rc != kInfOk || got != n || (n && std::memcmp(o.data(), d.data(), n) != 0)) {
      if (++bad < 5) std::printf("FAIL it %d n %zu level %d strategy %d rc %d got %u\n", it, n, level, strategy, rc, got);
    }
    // the CRC split over 64 chunks and recombined, as the device does
    const uint32_t want = (uint32_t)crc32(0, d.data(), (uInt)n);
    const size_t chunk = (n + 63) / 64;
    uint32_t all = 0;
    for (int l = 0; l < 64; ++l) {
      const size_t b = std::min(n, l * chunk), e = std::min(n, b + chunk);
      const uint32_t part = (uint32_t)crc32(0, d.data() + b, (uInt)(e - b));
      all ^= crc_shift(part, n - e);
    }
    if (all != want && ++crc_bad < 5) std::printf("CRC FAIL it %d n %zu\n", it, n);
    if (!c.empty()) {  // a flipped bit: any status, in bounds
      std::vector<uint8_t> cc = c;
      cc[rng() % cc.size()] ^= (uint8_t)(1u << (rng() % 8));
      inflate_raw<HostLanes>(cc.data(), (uint32_t)cc.size(), o.data(), (uint32_t)n, &got, *t);
    }
    if (c.size() > 2) inflate_raw<HostLanes>(c.data(), (uint32_t)c.size() / 2, o.data(), (uint32_t)n, &got, *t);
    if (n > 1) {  // too small an output
      const int r2 = inflate_raw<HostLanes>(c.data(), (uint32_t)c.size(), o.data(), (uint32_t)n - 1, &got, *t);
      if (r2 != kInfOverflow && ++bad < 5) std::printf("FAIL it %d: short output gave %d\n", it, r2);
    }
  }
  // CRC table entries agree with zlib's single-byte CRCs
  for (uint32_t i = 0; i < 256; ++i) {
    const uint8_t byte = (uint8_t)i;
    // crc32 of one byte = ~(table[~0 ^ byte & 0xff] ^ (~0 >> 8))
    const uint32_t c = ~(crc32_entry((0xFFu ^ byte) & 0xFFu) ^ (0xFFFFFFFFu >> 8));
    if (c != (uint32_t)crc32(0, &byte, 1) && ++crc_bad < 5) std::printf("CRC table FAIL %u\n", i);
  }
  delete t;
  std::printf("inflate: %d bad of %d; crc: %d bad\n", bad, iters, crc_bad);
  return bad || crc_bad ? 1 : 0;
}
