// Developer micro-benchmark (not shipped): where a caller shard's "decode"
// time goes — BGZF inflate alone, BAM record decode, and the caller's Read
// copies — over one window of a BAM, single-threaded.
// usage: decode_bench <bam> <chrom> <beg> <end> [passes]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "bam.h"
#include "bgzf.h"

using namespace fcsg;
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const std::string bam = argv[1], chrom = argv[2];
  const long beg = atol(argv[3]), end = atol(argv[4]);
  const int passes = argc > 5 ? atoi(argv[5]) : 3;
  for (int pass = 0; pass < passes; ++pass) {
    double t0 = now();
    BamReader rd(bam);
    const int tid = rd.header().ref_index(chrom);
    const uint64_t off = BamIndex(bam + ".bai").seek_offset(tid, beg);
    const double t_open = now() - t0;
    // inflate only: a second reader over the same blocks
    BgzfReader bz(bam);
    bz.seek(off);
    std::vector<uint8_t> sink(1 << 16);
    t0 = now();
    size_t bytes = 0;
    // as many bytes as the record pass reads (measured below); first pass: until end of window estimate
    rd.seek(off);
    BamRecord r;
    size_t n = 0, kept = 0;
    const uint64_t v0 = rd.tell();
    double t1 = now();
    std::vector<uint64_t> ends;
    while (rd.next(r)) {
      if (r.ref_id > tid || r.pos >= end) break;
      ++n;
    }
    const double t_decode = now() - t1;
    const uint64_t v1 = rd.tell();
    // inflate the same compressed range
    t1 = now();
    while ((bz.tell() >> 16) < (v1 >> 16)) {
      const size_t got = bz.read(sink.data(), sink.size());
      if (!got) break;
      bytes += got;
    }
    const double t_inflate = now() - t1;
    // decode + the caller's per-read copies (load_reads_one)
    rd.seek(off);
    t1 = now();
    struct Read {
      int64_t pos, end;
      std::vector<uint32_t> cigar;
      std::string seq;
      std::vector<uint8_t> qual;
      int mapq;
      std::string bi, bd;
    };
    std::vector<Read> out;
    while (rd.next(r)) {
      if (r.ref_id > tid || r.pos >= end) break;
      if (r.end() <= beg) continue;
      Read x;
      x.pos = r.pos;
      x.end = r.end();
      x.cigar = std::move(r.cigar);
      x.seq = std::move(r.seq);
      x.qual = std::move(r.qual);
      x.mapq = r.mapq;
      r.get_aux_string("BI", x.bi);
      r.get_aux_string("BD", x.bd);
      out.push_back(std::move(x));
      ++kept;
    }
    const double t_reads = now() - t1;
    std::printf("pass %d: %zu records (%zu kept), %.1f MB inflated, compressed %.1f MB; open %.4f s, inflate %.4f s, "
                "decode %.4f s, decode+reads %.4f s\n",
                pass, n, kept, bytes / 1e6, ((v1 >> 16) - (v0 >> 16)) / 1e6, t_open, t_inflate, t_decode, t_reads);
    (void)t0;
  }
  return 0;
}
