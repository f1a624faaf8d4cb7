#include "caller.h"

#include <sys/resource.h>
#include <time.h>

#include <algorithm>
#include <array>
#include <charconv>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <utility>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string_view>
#include <tuple>
#include <type_traits>

#include "bam.h"
#include "bam_input.h"
#include "common.h"
#include "fcship.h"
#include "gatk_prep.h"
#include "hugebuf.h"

namespace fcsg {

void CallerStats::add(const CallerStats& o) {
  reads += o.reads;
  regions += o.regions;
  pairs += o.pairs;
  cells += o.cells;
  calls += o.calls;
  device_passes += o.device_passes;
  decode_passes += o.decode_passes;
  inflate_gpu_chunks += o.inflate_gpu_chunks;
  inflate_host_chunks += o.inflate_host_chunks;
  cpu_seconds += o.cpu_seconds;
  for (int k = 0; k < 4; ++k) faults[k] += o.faults[k];
  rescued += o.rescued;
  seconds += o.seconds;
  phmm_seconds += o.phmm_seconds;
  phmm_device_seconds += o.phmm_device_seconds;
  rescue_device_seconds += o.rescue_device_seconds;
  decode_seconds += o.decode_seconds;
  pileup_seconds += o.pileup_seconds;
  region_seconds += o.region_seconds;
  genotype_seconds += o.genotype_seconds;
  output_seconds += o.output_seconds;
  helped_tasks += o.helped_tasks;
  helped_seconds += o.helped_seconds;
  helped_cpu_seconds += o.helped_cpu_seconds;
}

namespace {

// A read of the window: its CIGAR, bases, qualities and BI / BD strings live
// in the window's HugeSlab (no per-read heap blocks).
template <typename T>
struct View {
  const T* p = nullptr;
  size_t n = 0;
  const T* begin() const { return p; }
  const T* end() const { return p + n; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const T& operator[](size_t i) const { return p[i]; }
};
struct Read {
  int32_t pos = 0;
  int64_t end = 0;
  View<uint32_t> cigar;
  std::string_view seq;
  View<uint8_t> qual;
  int mapq = 0;
  std::string_view bi, bd;
};
static_assert(std::is_trivially_copyable_v<Read>, "Read lives in a HugeVec");

// window chunks of this thread inflated on the GPU / on the host (gpu.bam_inflate)
thread_local int64_t tl_inflate_gpu = 0, tl_inflate_host = 0;

void load_reads_one(const std::string& bam, const std::string& chrom, int64_t beg, int64_t end,
                    const CallerOptions& opt, HugeSlab& slab, HugeVec<Read>& out) {
  BamReader rd(bam);
  struct Count {
    const BamReader& r;
    ~Count() {
      tl_inflate_gpu += r.device_chunks();
      tl_inflate_host += r.host_chunks();
    }
  } count{rd};
  const int tid = rd.header().ref_index(chrom);
  if (tid < 0) return;
  const std::string bai = bam_index_path(bam);
  if (!bai.empty()) {
    const BamIndex ix(bai);
    const uint64_t off = ix.seek_offset(tid, beg);
    if (opt.gpu_inflate) {
      // the window's compressed span by the BAI's linear index at its end,
      // plus the reads that start in that last 16 kb window (at 30x about 0.4
      // MiB compressed; 1 MiB of margin)
      const uint64_t e = ix.seek_offset(tid, end);
      rd.use_device(opt.gpu, e > off ? (size_t)((e >> 16) - (off >> 16)) + (1 << 20) : 0);
    }
    if (off) rd.seek(off);
  } else if (opt.gpu_inflate) {
    rd.use_device(opt.gpu, 0);
  }
  // fields read straight from the raw record (decode_bam_record's layout),
  // filters applied before SEQ / QUAL are decoded
  auto get32 = [](const uint8_t* q) {
    int32_t v;
    std::memcpy(&v, q, 4);
    return v;
  };
  auto get16 = [](const uint8_t* q) {
    uint16_t v;
    std::memcpy(&v, q, 2);
    return v;
  };
  const uint8_t* p;
  size_t n;
  std::string tag;
  while (rd.next_raw(p, n)) {
    const int32_t ref_id = get32(p), pos = get32(p + 4);
    if (ref_id < tid) continue;
    if (ref_id > tid || pos >= end) break;
    const uint8_t l_name = p[8], mapq = p[9];
    const uint16_t n_cigar = get16(p + 12), flag = get16(p + 14);
    const int32_t l_seq = get32(p + 16);
    const size_t kc = 32 + (size_t)l_name, ks = kc + 4 * (size_t)n_cigar, kq = ks + (size_t)(l_seq + 1) / 2,
                 ka = kq + (size_t)l_seq;
    if (l_seq < 0 || ka > n) throw formatError("truncated BAM record");
    if (flag & (kUnmapped | kSecondary | kQcFail | kDuplicate | kSupplementary)) continue;
    if (mapq < opt.min_mapq || n_cigar == 0) continue;
    if (l_seq > 0 && p[kq] == 0xff) continue;  // QUAL absent
    int64_t rlen = 0;
    for (uint16_t i = 0; i < n_cigar; ++i) {
      const uint32_t c = (uint32_t)get32(p + kc + 4 * i);
      const CigarOp op = cigar_op(c);
      if (op == kM || op == kD || op == kN || op == kEq || op == kX) rlen += cigar_len(c);
    }
    const int64_t e = pos + rlen;
    if (e <= beg) continue;
    Read& x = out.emplace_back();
    x.pos = pos;
    x.end = e;
    uint8_t* m = slab.alloc(4 * (size_t)n_cigar + 2 * (size_t)l_seq, 4);
    std::memcpy(m, p + kc, 4 * (size_t)n_cigar);
    x.cigar = {reinterpret_cast<const uint32_t*>(m), n_cigar};
    m += 4 * (size_t)n_cigar;
    decode_bam_seq(p + ks, l_seq, reinterpret_cast<char*>(m));
    x.seq = std::string_view(reinterpret_cast<const char*>(m), (size_t)l_seq);
    std::memcpy(m + l_seq, p + kq, (size_t)l_seq);
    x.qual = {m + l_seq, (size_t)l_seq};
    x.mapq = mapq;
    for (int t = 0; t < 2; ++t) {
      if (!bam_aux_string(p + ka, n - ka, t ? "BD" : "BI", tag)) continue;
      char* c = reinterpret_cast<char*>(slab.alloc(tag.size(), 1));
      std::memcpy(c, tag.data(), tag.size());
      (t ? x.bd : x.bi) = std::string_view(c, tag.size());
    }
  }
}

// Reads of the window from every part of the sample, in coordinate order
// (parts of a `--disable-merge` alignment are each sorted).
void load_reads(const std::vector<std::string>& bams, const std::string& chrom, int64_t beg, int64_t end,
                const CallerOptions& opt, HugeSlab& slab, HugeVec<Read>& out) {
  for (const std::string& b : bams) load_reads_one(b, chrom, beg, end, opt, slab, out);
  if (bams.size() > 1)
    std::stable_sort(out.begin(), out.end(), [](const Read& a, const Read& b) { return a.pos < b.pos; });
}

struct Allele {
  int64_t pos;  // 0-based anchor
  std::string ref, alt;
  bool operator<(const Allele& o) const { return std::tie(pos, ref, alt) < std::tie(o.pos, o.ref, o.alt); }
  int64_t ref_end() const { return pos + (int64_t)ref.size(); }
};

struct Pileup {
  int64_t wb = 0;
  HugeArray<int> depth, events;
  // allele events of the reads — SNVs as packed (pos, ref, alt) keys, indels
  // as Alleles — then (finish_support) sorted and counted: the support of
  // each distinct allele in (pos, ref, alt) order
  HugeVec<uint64_t> snv_events;
  std::vector<Allele> indel_events;
  std::vector<std::pair<Allele, int>> support;
  // GVCF reference model: per position, sum over bases of log10 P(base | 0/0,
  // 0/1, 1/1) with 1 = <NON_REF> (any other base)
  HugeArray<double> gl;  // 3 per position; empty unless GVCF
};

// log10 P(base | genotype) per base quality: [q][0] ref base under 0/0 (1 - e),
// [q][1] any base under 0/1 (0.5 (1 - e) + 0.5 e / 3), [q][2] non-ref base
// under 0/0 (e / 3); a ref base under 1/1 is e / 3, a non-ref base 1 - e.
struct RefModel {
  double t[94][3];
  RefModel() {
    for (int q = 0; q < 94; ++q) {
      const double e = std::min(0.75, std::pow(10.0, -q / 10.0));
      t[q][0] = std::log10(1.0 - e);
      t[q][1] = std::log10(0.5 * (1.0 - e) + 0.5 * e / 3.0);
      t[q][2] = std::log10(e / 3.0);
    }
  }
};
const RefModel& ref_model() {
  static const RefModel m;
  return m;
}

inline uint64_t snv_key(int64_t pos, char ref, char alt) {
  return ((uint64_t)pos << 16) | ((uint64_t)(uint8_t)ref << 8) | (uint8_t)alt;
}

// Walks every read's CIGAR once: depth, mismatch/indel events and allele support.
void build_pileup(const std::string& ref, const HugeVec<Read>& reads, int min_bq, Pileup& pu) {
  const int64_t n = (int64_t)pu.depth.size();
  const int64_t wb = pu.wb, we = pu.wb + n;
  auto in = [&](int64_t p) { return p >= wb && p < we; };
  const RefModel& M = ref_model();
  int* depth = pu.depth.data();
  int* events = pu.events.data();
  double* gl = pu.gl.empty() ? nullptr : pu.gl.data();
  for (const Read& rd : reads) {
    int64_t rp = rd.pos;
    size_t q = 0;
    for (uint32_t c : rd.cigar) {
      const uint32_t len = cigar_len(c);
      switch (cigar_op(c)) {
        case kM: case kEq: case kX: {
          // only the bases inside the window
          const int64_t lo = std::max<int64_t>(rp, wb), hi = std::min<int64_t>(rp + len, we);
          for (int64_t p = lo; p < hi; ++p) {
            const size_t qi = q + (size_t)(p - rp);
            const uint8_t bq = rd.qual[qi];
            if (bq < min_bq) continue;
            ++depth[p - wb];
            const char b = rd.seq[qi], r = ref[p];
            const bool nonref = b != r && r != 'N' && b != 'N';
            if (nonref) {
              ++events[p - wb];
              pu.snv_events.emplace_back() = snv_key(p, r, b);
            }
            if (gl) {
              const double* t = M.t[std::min<int>(bq, 93)];
              double* g = gl + 3 * (p - wb);
              g[0] += t[nonref ? 2 : 0];
              g[1] += t[1];
              g[2] += t[nonref ? 0 : 2];
            }
          }
          rp += len;
          q += len;
          break;
        }
        case kI:
          if (rp > rd.pos && in(rp - 1)) {
            ++events[rp - 1 - wb];
            pu.indel_events.push_back({rp - 1, std::string(1, ref[rp - 1]), std::string(1, ref[rp - 1]).append(rd.seq.substr(q, len))});
          }
          q += len;
          break;
        case kD:
          if (rp > rd.pos && in(rp - 1) && rp + len <= (int64_t)ref.size()) {
            ++events[rp - 1 - wb];
            pu.indel_events.push_back({rp - 1, ref.substr(rp - 1, len + 1), std::string(1, ref[rp - 1])});
          }
          for (int64_t p = std::max<int64_t>(rp, wb), hi = std::min<int64_t>(rp + len, we); p < hi; ++p) ++depth[p - wb];
          rp += len;
          break;
        case kN: rp += len; break;
        case kS: q += len; break;
        default: break;
      }
    }
  }
}

// The distinct alleles of the pileup's events seen in at least two reads
// (the least support a candidate allele needs), with their read counts, in
// (pos, ref, alt) order: the SNV keys sort as integers (a one-base REF and
// ALT compare as their bytes), the indels as Alleles, and the two runs merge
// (an indel never equals an SNV: its REF or ALT is longer than one base).
void finish_support(Pileup& pu) {
  std::sort(pu.snv_events.begin(), pu.snv_events.end());
  std::sort(pu.indel_events.begin(), pu.indel_events.end());
  pu.support.clear();
  size_t i = 0, j = 0;
  const size_t ns = pu.snv_events.size(), ni = pu.indel_events.size();
  auto next_snv = [&] {  // skip SNVs seen once
    while (i < ns && (i + 1 >= ns || pu.snv_events[i + 1] != pu.snv_events[i])) ++i;
  };
  auto next_indel = [&] {
    while (j < ni && (j + 1 >= ni || pu.indel_events[j] < pu.indel_events[j + 1])) ++j;
  };
  next_snv();
  next_indel();
  while (i < ns || j < ni) {
    if (i < ns) {
      const uint64_t k = pu.snv_events[i];
      Allele a{(int64_t)(k >> 16), std::string(1, (char)((k >> 8) & 0xff)), std::string(1, (char)(k & 0xff))};
      if (j >= ni || a < pu.indel_events[j]) {
        size_t e = i;
        while (e < ns && pu.snv_events[e] == k) ++e;
        pu.support.emplace_back(std::move(a), (int)(e - i));
        i = e;
        next_snv();
        continue;
      }
    }
    Allele& a = pu.indel_events[j];
    size_t e = j + 1;
    while (e < ni && !(a < pu.indel_events[e])) ++e;
    pu.support.emplace_back(std::move(a), (int)(e - j));
    j = e;
    next_indel();
  }
  pu.snv_events = HugeVec<uint64_t>();
  std::vector<Allele>().swap(pu.indel_events);
}

// Query slice [qs, qe) of the read whose bases align inside [rb, re) (inserted
// bases go with their left anchor); soft clips excluded.  false if empty.
bool clip_to_window(const Read& rd, int64_t rb, int64_t re, size_t& qs, size_t& qe) {
  // per CIGAR op: the query span whose anchors (the reference base of an M
  // base; an inserted base's left neighbour) fall inside [rb, re); anchors
  // never decrease along the read, so the taken bases form one slice
  int64_t rp = rd.pos, anchor = rd.pos - 1;
  size_t q = 0;
  bool started = false;
  qs = qe = 0;
  auto take = [&](size_t a, size_t b) {  // query [a, b) taken
    if (!started) qs = a, started = true;
    qe = b;
  };
  for (uint32_t c : rd.cigar) {
    const uint32_t len = cigar_len(c);
    switch (cigar_op(c)) {
      case kM: case kEq: case kX: {
        const int64_t lo = std::max<int64_t>(rp, rb), hi = std::min<int64_t>(rp + len, re);
        if (lo < hi) take(q + (size_t)(lo - rp), q + (size_t)(hi - rp));
        if (len) anchor = rp + len - 1;
        rp += len;
        q += len;
        break;
      }
      case kI:
        if (len && anchor >= rb && anchor < re) take(q, q + len);
        q += len;
        break;
      case kD: case kN: rp += len; anchor = rp - 1; break;
      case kS: q += len; break;
      default: break;
    }
  }
  return started && qe > qs;
}

// A region's prepared reads in one arena: per read the five rows gatk_prep
// writes (bases, base_q, ins_q, del_q, gcp; n bytes each) back to back, so
// preparing a read costs no allocation.
struct PreparedSet {
  std::vector<uint8_t> buf;
  std::vector<std::pair<size_t, int32_t>> at;  // per read: offset in buf, length
  size_t size() const { return at.size(); }
  bool empty() const { return at.empty(); }
  uint8_t* add(int32_t n) {
    at.emplace_back(buf.size(), n);
    buf.resize(buf.size() + 5 * (size_t)n);
    return buf.data() + at.back().first;
  }
  int32_t len(size_t i) const { return at[i].second; }
  const uint8_t* row(size_t i, int k) const { return buf.data() + at[i].first + (size_t)k * (size_t)at[i].second; }
};

struct Region {
  int64_t beg = 0, end = 0;  // reference window [beg, end)
  std::vector<Allele> cands;
  std::vector<std::string> haps;
  std::vector<uint32_t> hap_mask;  // bit c: haplotype carries candidate c
  PreparedSet reads[2];                // [0] sample / tumor, [1] normal
  std::vector<double> lik[2];          // read-major log10 likelihoods
};

void build_haplotypes(const std::string& ref, Region& g) {
  const int k = (int)g.cands.size();
  for (uint32_t mask = 0; mask < (1u << k); ++mask) {
    std::vector<const Allele*> on;
    for (int c = 0; c < k; ++c)
      if (mask >> c & 1) on.push_back(&g.cands[c]);
    std::sort(on.begin(), on.end(), [](const Allele* a, const Allele* b) { return a->pos < b->pos; });
    bool ok = true;
    for (size_t i = 1; i < on.size(); ++i)
      if (on[i]->pos < on[i - 1]->ref_end()) ok = false;  // overlapping alleles cannot share a haplotype
    if (!ok) continue;
    std::string h;
    int64_t p = g.beg;
    for (const Allele* a : on) {
      h.append(ref, p, a->pos - p);
      h += a->alt;
      p = a->ref_end();
    }
    h.append(ref, p, g.end - p);
    g.haps.push_back(std::move(h));
    g.hap_mask.push_back(mask);
  }
}

double log10_add(double a, double b) {
  const double m = std::max(a, b);
  if (m == -INFINITY) return m;
  return m + std::log10(std::pow(10.0, a - m) + std::pow(10.0, b - m));
}

// Per read: best log10 likelihood among haplotypes with / without candidate c.
void allele_lik(const Region& g, int s, int c, std::vector<double>& la, std::vector<double>& lr) {
  const size_t nr = g.reads[s].size(), nh = g.haps.size();
  la.assign(nr, -INFINITY);
  lr.assign(nr, -INFINITY);
  for (size_t r = 0; r < nr; ++r)
    for (size_t h = 0; h < nh; ++h) {
      const double v = g.lik[s][r * nh + h];
      if (g.hap_mask[h] >> c & 1) la[r] = std::max(la[r], v);
      else lr[r] = std::max(lr[r], v);
    }
}

void dump_region(std::FILE* f, const Region& g, int s) {
  const int32_t nr = (int32_t)g.reads[s].size(), nh = (int32_t)g.haps.size();
  std::fwrite("RGN1", 1, 4, f);
  std::fwrite(&nr, 4, 1, f);
  std::fwrite(&nh, 4, 1, f);
  for (size_t i = 0; i < g.reads[s].size(); ++i) {
    const int32_t L = g.reads[s].len(i);
    std::fwrite(&L, 4, 1, f);
    std::fwrite(g.reads[s].row(i, 0), 1, 5 * (size_t)L, f);  // the five rows, in dump order
  }
  for (const std::string& h : g.haps) {
    const int32_t L = (int32_t)h.size();
    std::fwrite(&L, 4, 1, f);
    std::fwrite(h.data(), 1, L, f);
  }
  std::fwrite(g.lik[s].data(), 8, g.lik[s].size(), f);
}

// Device passes of concurrent shard threads merged into one (group commit).
// Each shard of `htc` / `mutect2` batches its own regions, so at the C4 shape
// (31 Mbp per GPU in 32 shards) a pass is ~87K pairs, and the per-pass fixed
// work (schedule sort, class launches, rescue) holds the device-effective rate
// to about half of a 1M-pair pass.  Shard threads hand their region lists to
// the combiner of their (device, rescue) slot; the oldest waiting request
// leads: it gathers until every active shard thread of the slot is waiting,
// its window (`gpu.phmm.combine_ms`) ends or the pass holds `max_pairs`, then
// runs ONE fcs_phmm_compute_regions over the concatenated region list (each
// region keeps its own output matrix, so results are bitwise those of separate
// passes) while later requests queue for the next pass.  A waiting thread
// yields its CPU to the shards still building regions.
class PassCombiner {
 public:
  struct Req {
    const std::vector<fcs_phmm_region>* regs = nullptr;
    int64_t pairs = 0;
    int rc = FCS_OK;
    std::string err;
    bool done = false, led = false;
    double dev_ms = 0, res_ms = 0;
    int64_t rescued = 0;
  };
  void enter() {
    std::lock_guard<std::mutex> g(m_);
    ++active_;
  }
  void leave() {
    std::lock_guard<std::mutex> g(m_);
    --active_;
    cv_.notify_all();
  }
  void run(Req& r, const fcs_phmm_opts& o, int window_ms, int64_t max_pairs) {
    std::unique_lock<std::mutex> lk(m_);
    q_.push_back(&r);
    cv_.notify_all();
    // system_clock: waits on it are pthread_cond_timedwait, which ThreadSanitizer
    // follows (a steady_clock wait_until is pthread_cond_clockwait in this
    // libstdc++, which GCC 11's TSAN does not intercept: false double locks)
    const auto deadline = std::chrono::system_clock::now() + std::chrono::milliseconds(window_ms);
    while (!r.done) {
      if (busy_ || q_.front() != &r) {
        cv_.wait(lk);
        continue;
      }
      auto ready = [&] {
        int64_t pairs = 0;
        for (const Req* x : q_) pairs += x->pairs;
        return (int)q_.size() >= active_ || pairs >= max_pairs;
      };
      while (!ready() && cv_.wait_until(lk, deadline) != std::cv_status::timeout) {
      }
      std::vector<Req*> take;
      int64_t tp = 0;
      while (!q_.empty() && (take.empty() || tp + q_.front()->pairs <= max_pairs)) {
        tp += q_.front()->pairs;
        take.push_back(q_.front());
        q_.pop_front();
      }
      busy_ = true;
      lk.unlock();
      // nothing may leave this section by exception: the taken requests must be
      // marked done and busy_ cleared, or every waiter of the slot blocks forever
      int rc = FCS_OK;
      std::string err;
      double dev = 0, res = 0;
      int64_t nres = 0;
      try {
        std::vector<fcs_phmm_region> all;
        for (const Req* x : take) all.insert(all.end(), x->regs->begin(), x->regs->end());
        rc = fcs_phmm_compute_regions(all.data(), (int32_t)all.size(), &o);
        if (rc != FCS_OK) err = fcs_last_error();
        if (rc == FCS_OK) {
          if (fcs_phmm_last_rescued(&nres) != FCS_OK) nres = 0;
          if (fcs_phmm_last_device_ms(&dev, &res) != FCS_OK) dev = res = 0;
        }
      } catch (const std::exception& e) {
        rc = FCS_ERR_INVALID;
        err = std::string("[E::fcsg] merged PairHMM pass: ") + e.what();
      } catch (...) {
        rc = FCS_ERR_INVALID;
        err = "[E::fcsg] merged PairHMM pass: unknown exception";
      }
      lk.lock();
      for (Req* x : take) x->rc = rc, x->err = err, x->done = true;
      r.led = true, r.dev_ms = dev, r.res_ms = res, r.rescued = nres;
      busy_ = false;
      cv_.notify_all();
    }
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<Req*> q_;
  bool busy_ = false;
  int active_ = 0;
};

PassCombiner& pass_combiner(int gpu, bool rescue) {
  static std::mutex m;
  static std::map<std::pair<int, bool>, std::unique_ptr<PassCombiner>> slots;
  std::lock_guard<std::mutex> g(m);
  auto& c = slots[{gpu, rescue}];
  if (!c) c = std::make_unique<PassCombiner>();
  return *c;
}

// A shard thread counts as active on its slot's combiner while it calls.
struct CombinerScope {
  PassCombiner* c;
  explicit CombinerScope(const CallerOptions& opt)
      : c(opt.combine_ms > 0 ? &pass_combiner(opt.gpu, opt.fp64_rescue) : nullptr) {
    if (c) c->enter();
  }
  ~CombinerScope() {
    if (c) c->leave();
  }
  CombinerScope(const CombinerScope&) = delete;
  CombinerScope& operator=(const CombinerScope&) = delete;
};

// One device pass over a batch of regions (both read sets in Mutect2 mode).
void run_phmm(std::vector<std::unique_ptr<Region>>& batch, const CallerOptions& opt, CallerStats& st, std::FILE* dump) {
  std::vector<std::vector<fcs_phmm_read>> rv;
  std::vector<std::vector<fcs_phmm_hap>> hv(batch.size());
  std::vector<fcs_phmm_region> regs;
  rv.reserve(2 * batch.size());
  for (size_t i = 0; i < batch.size(); ++i) {
    Region& g = *batch[i];
    for (const std::string& h : g.haps) hv[i].push_back({reinterpret_cast<const uint8_t*>(h.data()), (int32_t)h.size()});
    for (int s = 0; s < 2; ++s) {
      g.lik[s].assign(g.reads[s].size() * g.haps.size(), 0.0);
      if (g.reads[s].empty()) continue;
      rv.emplace_back();
      const PreparedSet& ps = g.reads[s];
      int64_t hap_bases = 0;
      for (const std::string& h : g.haps) hap_bases += (int64_t)h.size();
      for (size_t r = 0; r < ps.size(); ++r) {
        rv.back().push_back({ps.row(r, 0), ps.row(r, 1), ps.row(r, 2), ps.row(r, 3), ps.row(r, 4), ps.len(r)});
        st.cells += (int64_t)ps.len(r) * hap_bases;
      }
      regs.push_back({rv.back().data(), (int32_t)rv.back().size(), hv[i].data(), (int32_t)hv[i].size(),
                      g.lik[s].data()});
      st.pairs += (int64_t)g.reads[s].size() * (int64_t)g.haps.size();
    }
  }
  fcs_phmm_opts o;
  fcs_phmm_opts_default(&o);
  o.device = opt.gpu;
  o.use_fp64_rescue = opt.fp64_rescue ? 1 : 0;
  const uint64_t t0 = now_us();
  if (opt.combine_ms > 0) {
    PassCombiner::Req r;
    r.regs = &regs;
    for (const fcs_phmm_region& g : regs) r.pairs += (int64_t)g.n_reads * g.n_haps;
    pass_combiner(opt.gpu, opt.fp64_rescue).run(r, o, opt.combine_ms, opt.combine_max_pairs);
    st.phmm_seconds += (now_us() - t0) / 1e6;
    if (r.rc != FCS_OK) throw failedCommand(r.err);
    if (r.led) {  // the pass's device time and rescues count once, on the thread that ran it
      ++st.device_passes;
      st.rescued += r.rescued;
      st.phmm_device_seconds += r.dev_ms / 1e3;
      st.rescue_device_seconds += r.res_ms / 1e3;
    }
  } else {
    const int rc = fcs_phmm_compute_regions(regs.data(), (int32_t)regs.size(), &o);
    st.phmm_seconds += (now_us() - t0) / 1e6;
    ++st.device_passes;
    if (rc != FCS_OK) throw failedCommand(std::string(fcs_last_error()));
    int64_t nres = 0;
    if (fcs_phmm_last_rescued(&nres) == FCS_OK) st.rescued += nres;
    double dev_ms = 0, res_ms = 0;
    if (fcs_phmm_last_device_ms(&dev_ms, &res_ms) == FCS_OK) {
      st.phmm_device_seconds += dev_ms / 1e3;
      st.rescue_device_seconds += res_ms / 1e3;
    }
  }
  if (dump)
    for (const auto& g : batch)
      for (int s = 0; s < 2; ++s)
        if (!g->reads[s].empty()) dump_region(dump, *g, s);
}

// Germline diploid genotyping of each candidate allele of a region.
void genotype_germline(const Region& g, const CallerOptions& opt, int64_t own_beg, int64_t own_end,
                       const std::string& chrom, std::vector<VcfRecord>& calls) {
  static const double prior[3] = {std::log10(1.0 - 1.5e-3), std::log10(1e-3), std::log10(5e-4)};
  std::vector<double> la, lr;
  for (size_t c = 0; c < g.cands.size(); ++c) {
    const Allele& a = g.cands[c];
    if (a.pos < own_beg || a.pos >= own_end) continue;
    allele_lik(g, 0, (int)c, la, lr);
    double gl[3] = {0, 0, 0};
    int ad_ref = 0, ad_alt = 0;
    for (size_t r = 0; r < la.size(); ++r) {
      gl[0] += lr[r];
      gl[2] += la[r];
      gl[1] += log10_add(la[r], lr[r]) - std::log10(2.0);
      if (la[r] - lr[r] > 0.2) ++ad_alt;
      else if (lr[r] - la[r] > 0.2) ++ad_ref;
    }
    double post[3], mx = -INFINITY;
    for (int k = 0; k < 3; ++k) mx = std::max(mx, post[k] = gl[k] + prior[k]);
    double norm = -INFINITY;
    for (int k = 0; k < 3; ++k) norm = log10_add(norm, post[k]);
    const int gt = (int)(std::max_element(post, post + 3) - post);
    const double qual = std::min(-10.0 * (post[0] - norm), 9999.0);
    if (gt == 0 || qual < opt.min_qual) continue;
    const double glmax = std::max({gl[0], gl[1], gl[2]});
    int pl[3];
    for (int k = 0; k < 3; ++k) pl[k] = (int)std::lround(-10.0 * (gl[k] - glmax));
    int sorted[3] = {pl[0], pl[1], pl[2]};
    std::sort(sorted, sorted + 3);
    const int gq = std::min(99, sorted[1]);
    VcfRecord rec;
    rec.chrom = chrom;
    rec.pos = a.pos + 1;
    rec.ref = a.ref;
    rec.alts = {a.alt};
    rec.qual = qual;
    rec.info = "DP=" + std::to_string(la.size());
    rec.format = "GT:AD:DP:GQ:PL";
    std::string pls = std::to_string(pl[0]) + "," + std::to_string(pl[1]) + "," + std::to_string(pl[2]);
    std::string ad = std::to_string(ad_ref) + "," + std::to_string(ad_alt);
    if (opt.gvcf) {
      // <NON_REF> as a third allele [EXT stand-in for GATK's non-ref likelihoods]:
      // each read's likelihood under it is its worst haplotype's; PLs of the six
      // genotypes (0/0 0/1 1/1 0/2 1/2 2/2) from the same diploid model
      const size_t nh = g.haps.size();
      double g6[6] = {gl[0], gl[1], gl[2], 0, 0, 0};
      for (size_t r = 0; r < la.size(); ++r) {
        double ln = INFINITY;
        for (size_t h = 0; h < nh; ++h) ln = std::min(ln, g.lik[0][r * nh + h]);
        g6[3] += log10_add(lr[r], ln) - std::log10(2.0);
        g6[4] += log10_add(la[r], ln) - std::log10(2.0);
        g6[5] += ln;
      }
      const double m6 = *std::max_element(g6, g6 + 6);
      pls.clear();
      for (int k = 0; k < 6; ++k) pls += (k ? "," : "") + std::to_string((int)std::lround(-10.0 * (g6[k] - m6)));
      rec.alts.push_back("<NON_REF>");
      ad += ",0";
    }
    rec.samples = {std::string(gt == 1 ? "0/1" : "1/1") + ":" + ad + ":" + std::to_string(la.size()) + ":" +
                   std::to_string(gq) + ":" + pls};
    calls.push_back(rec);
  }
}

// Mutect2-style tumor/normal test of each candidate allele.
void genotype_somatic(const Region& g, const CallerOptions& opt, int64_t own_beg, int64_t own_end,
                      const std::string& chrom, std::vector<VcfRecord>& calls) {
  std::vector<double> ta, tr, na, nr;
  for (size_t c = 0; c < g.cands.size(); ++c) {
    const Allele& a = g.cands[c];
    if (a.pos < own_beg || a.pos >= own_end) continue;
    allele_lik(g, 0, (int)c, ta, tr);
    allele_lik(g, 1, (int)c, na, nr);
    int t_alt = 0, t_ref = 0, n_alt = 0, n_ref = 0;
    for (size_t r = 0; r < ta.size(); ++r) {
      if (ta[r] - tr[r] > 0.2) ++t_alt;
      else if (tr[r] - ta[r] > 0.2) ++t_ref;
    }
    for (size_t r = 0; r < na.size(); ++r) {
      if (na[r] - nr[r] > 0.2) ++n_alt;
      else if (nr[r] - na[r] > 0.2) ++n_ref;
    }
    if (t_alt == 0) continue;
    const double f = std::max(1e-3, (double)t_alt / std::max(1, t_alt + t_ref));
    double tlod = 0, nlod = 0;
    for (size_t r = 0; r < ta.size(); ++r)
      tlod += log10_add(std::log10(f) + ta[r], std::log10(1.0 - f) + tr[r]) - tr[r];
    for (size_t r = 0; r < na.size(); ++r) nlod += nr[r] - (log10_add(na[r], nr[r]) - std::log10(2.0));
    if (tlod < opt.tlod || nlod < opt.nlod) continue;
    VcfRecord rec;
    rec.chrom = chrom;
    rec.pos = a.pos + 1;
    rec.ref = a.ref;
    rec.alts = {a.alt};
    char info[96];
    std::snprintf(info, sizeof info, "TLOD=%.2f;NLOD=%.2f", tlod, nlod);
    rec.info = info;
    rec.format = "GT:AD:AF";
    char taf[32];
    std::snprintf(taf, sizeof taf, "%.3f", f);
    rec.samples = {"0/1:" + std::to_string(t_ref) + "," + std::to_string(t_alt) + ":" + taf,
                   "0/0:" + std::to_string(n_ref) + "," + std::to_string(n_alt) + ":0.000"};
    calls.push_back(rec);
  }
}

// Reference-confidence blocks of [beg, end) around this interval's calls
// (GATK --emitRefConfidence GVCF): every position not inside a call's REF span
// gets the hom-ref genotype likelihoods of its pileup (RefModel); runs of
// positions whose GQ falls in one band become one record
// "<NON_REF> END=..  GT:DP:GQ:MIN_DP:PL" with the block's median DP, minimum
// GQ / DP and element-wise minimum PLs.  Blocks are kept as plain numbers
// (GvcfBlock) and the output sequence as entries naming a block or a call:
// the GVCF's hundreds of thousands of block lines are formatted straight into
// the writer's buffer, never built as VcfRecord strings.
struct GvcfBlock {
  int64_t b, e;  // 0-based first / last position
  int dp, gq, mindp;
  int pl[3];
};
struct OutEntry {
  int32_t contig;  // reference contig index
  int32_t block;   // into the GvcfBlock list, or -1
  int64_t call;    // into the calls, or -1
  int64_t pos;     // 1-based POS
};

// std::lround of a phred-scaled likelihood difference (v >= 0, < 2^31): the
// truncation plus the exact fraction test rounds halves away from zero as
// lround does, at a quarter of its cost (emit_gvcf runs it 3 times a base)
inline int round_phred(double v) {
  const int r = (int)v;
  return r + (v - (double)r >= 0.5 ? 1 : 0);
}

void emit_gvcf(const Pileup& pu, int64_t beg, int64_t end, int contig, const std::vector<VcfRecord>& calls,
               size_t c0, HugeVec<GvcfBlock>& blocks, HugeVec<OutEntry>& out) {
  std::vector<size_t> ic;  // this interval's calls in POS order (stable)
  for (size_t i = c0; i < calls.size(); ++i) ic.push_back(i);
  std::stable_sort(ic.begin(), ic.end(), [&](size_t a, size_t b) { return calls[a].pos < calls[b].pos; });
  struct Block {
    int64_t b = -1, e = -1;
    int band = -1, gq = 99, mindp = 0;
    int pl[3] = {0, 0, 0};
  } blk;
  std::vector<int> dps;
  auto flush = [&] {
    if (blk.b < 0) return;
    std::nth_element(dps.begin(), dps.begin() + dps.size() / 2, dps.end());
    out.emplace_back() = {contig, (int32_t)blocks.size(), -1, blk.b + 1};
    blocks.emplace_back() = {blk.b, blk.e, dps[dps.size() / 2], blk.gq, blk.mindp, {blk.pl[0], blk.pl[1], blk.pl[2]}};
    dps.clear();
    blk = Block();
  };
  size_t ci = 0;
  int64_t covered = beg;  // positions below are inside an emitted call's REF span
  for (int64_t p = beg; p < end; ++p) {
    while (ci < ic.size() && calls[ic[ci]].pos - 1 <= p) {
      flush();
      const VcfRecord& c = calls[ic[ci]];
      out.emplace_back() = {contig, -1, (int64_t)ic[ci], c.pos};
      covered = std::max<int64_t>(covered, c.pos - 1 + (int64_t)c.ref.size());
      ++ci;
    }
    if (p < covered) continue;
    const int dp = pu.depth[p - pu.wb];
    const double* g = &pu.gl[3 * (p - pu.wb)];
    const double mx = std::max({g[0], g[1], g[2]});
    int pl[3];
    for (int k = 0; k < 3; ++k) pl[k] = round_phred(-10.0 * (g[k] - mx));
    const int gq = (pl[0] == 0) ? std::min(99, std::min(pl[1], pl[2])) : 0;
    const int band = gvcf_band(gq);
    if (blk.b < 0 || band != blk.band || p != blk.e + 1) {
      flush();
      blk.b = p;
      blk.band = band;
      blk.gq = gq;
      blk.mindp = dp;
      for (int k = 0; k < 3; ++k) blk.pl[k] = pl[k];
    }
    blk.e = p;
    blk.gq = std::min(blk.gq, gq);
    blk.mindp = std::min(blk.mindp, dp);
    for (int k = 0; k < 3; ++k) blk.pl[k] = std::min(blk.pl[k], pl[k]);
    dps.push_back(dp);
  }
  flush();
  for (; ci < ic.size(); ++ci) out.emplace_back() = {contig, -1, (int64_t)ic[ci], calls[ic[ci]].pos};
}

// One GVCF block line, as VcfRecord::append_line writes the record
// {chrom, b + 1, ".", REF, "<NON_REF>", ".", ".", "END=e + 1",
//  "GT:DP:GQ:MIN_DP:PL", "0/0:DP:GQ:MIN_DP:PL0,PL1,PL2"}.
// (GCC's -Wstringop-overflow cannot bound to_chars' result pointer here; the
// buffer holds the longest line, see its size)
#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wstringop-overflow"
#pragma GCC diagnostic ignored "-Warray-bounds"
void append_block_line(const std::string& chrom, char ref, const GvcfBlock& k, std::string& s) {
  char b[256 + 64];  // a short contig name + 2 x 20 + 6 x 11 digits + 60 literal bytes at most
  char* p = b;
  auto num = [&](int64_t v) { p = std::to_chars(p, b + sizeof b, v).ptr; };  // (gcc's: 2 digits a step)
  auto lit = [&](std::string_view t) {
    std::memcpy(p, t.data(), t.size());
    p += t.size();
  };
  if (chrom.size() <= 64) {
    lit(chrom);
  } else {
    s += chrom;
  }
  *p++ = '\t';
  num(k.b + 1);
  lit("\t.\t");
  *p++ = ref;
  lit("\t<NON_REF>\t.\t.\tEND=");
  num(k.e + 1);
  lit("\tGT:DP:GQ:MIN_DP:PL\t0/0:");
  num(k.dp);
  *p++ = ':';
  num(k.gq);
  *p++ = ':';
  num(k.mindp);
  *p++ = ':';
  num(k.pl[0]);
  *p++ = ',';
  num(k.pl[1]);
  *p++ = ',';
  num(k.pl[2]);
  *p++ = '\n';
  s.append(b, (size_t)(p - b));
}
#pragma GCC diagnostic pop

}  // namespace

int gvcf_band(int gq) {
  static const int bounds[] = {1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22,
                               23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44,
                               45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 70, 80, 90, 99};
  auto band = [&](int g) { return (int)(std::upper_bound(std::begin(bounds), std::end(bounds), g) - std::begin(bounds)); };
  // GQ is 0 .. 99 in emit_gvcf: a table; anything else by search
  static const auto lut = [&] {
    std::array<int, 100> t{};
    for (int g = 0; g < 100; ++g) t[g] = band(g);
    return t;
  }();
  return gq >= 0 && gq < 100 ? lut[gq] : band(gq);
}

namespace {
int64_t thread_faults() {
  struct rusage ru {};
  getrusage(RUSAGE_THREAD, &ru);
  return ru.ru_minflt;
}
double thread_cpu() {
  timespec ts{};
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return ts.tv_sec + ts.tv_nsec / 1e9;
}
}  // namespace

CallerStats call_intervals(const Reference& ref, const std::vector<std::string>& bams,
                           const std::vector<std::string>& normal_bams, const std::vector<Interval>& intervals_in,
                           const CallerOptions& opt, VcfWriter& out) {
  CallerStats st;
  const CombinerScope combiner(opt);
  const uint64_t t0 = now_us();
  const double cpu0 = thread_cpu();
  std::FILE* dump = opt.dump_path.empty() ? nullptr : std::fopen(opt.dump_path.c_str(), "ab");
  std::vector<VcfRecord> calls;
  HugeVec<GvcfBlock> blocks;  // GVCF mode: reference blocks and the output sequence
  HugeVec<OutEntry> gout;
  const std::vector<Interval>& intervals = intervals_in;
  std::vector<std::unique_ptr<Region>> pending;
  std::vector<std::tuple<int64_t, int64_t, std::string>> own;  // per pending region: owned range + chrom
  int64_t helped_faults = 0;
  auto flush = [&] {
    if (pending.empty()) return;
    if (interrupted()) throw interruptedError();
    if (opt.help_while_cold) {
      const uint64_t th = now_us();
      const double ch = thread_cpu();
      const int64_t fh = thread_faults();
      while (opt.help_while_cold()) ++st.helped_tasks;
      st.helped_seconds += (now_us() - th) / 1e6;
      st.helped_cpu_seconds += thread_cpu() - ch;
      helped_faults += thread_faults() - fh;
    }
    run_phmm(pending, opt, st, dump);
    const uint64_t tg = now_us();
    for (size_t i = 0; i < pending.size(); ++i) {
      const auto& [ob, oe, chrom] = own[i];
      if (opt.somatic) genotype_somatic(*pending[i], opt, ob, oe, chrom, calls);
      else genotype_germline(*pending[i], opt, ob, oe, chrom, calls);
    }
    st.genotype_seconds += (now_us() - tg) / 1e6;
    pending.clear();
    own.clear();
  };
  for (const Interval& iv : intervals) {
    if (interrupted()) throw interruptedError();
    const size_t c0 = calls.size();
    const int ci = ref.index(iv.chrom);
    if (ci < 0) throw invalidParam("interval contig " + iv.chrom + " is not in the reference");
    const std::string& seq = ref.contigs[ci].seq;
    const int64_t L = (int64_t)seq.size();
    const int64_t own_beg = std::max<int64_t>(0, iv.lb - 1), own_end = std::min<int64_t>(L, iv.ub);
    if (own_beg >= own_end) continue;
    // Active-site clusters (sites chained while the gap is <= padding) are the
    // connected components of the whole contig's site graph, so every shard
    // that sees a cluster must see all of it: the window around the shard's
    // own range grows until no cluster overlapping that range comes within
    // `padding` of a window edge (a site beyond the edge could chain on, and
    // the cluster's regions reach `padding` past its end sites).  Then the
    // regions, their candidates and reads, and so the likelihoods and calls,
    // do not depend on where gatk.ncontigs put the shard boundaries.
    int64_t ext_l = opt.max_region, ext_r = opt.max_region, wb = 0, we = 0;
    HugeVec<Read> reads[2];
    HugeSlab slab;  // the reads' bytes
    Pileup pu;
    std::vector<std::pair<int64_t, int64_t>> clusters;  // [first site, last site] overlapping the own range
    for (;;) {
      wb = std::max<int64_t>(0, own_beg - ext_l);
      we = std::min<int64_t>(L, own_end + ext_r);
      reads[0].clear();
      reads[1].clear();
      slab.clear();
      // ~0.2 reads per base at 30x of 150 bp: reserving address space (untouched
      // pages cost nothing) saves the vector's doubling copies
      for (int s = 0; s < (opt.somatic ? 2 : 1); ++s) reads[s].reserve((size_t)(we - wb) / 2);
      const uint64_t td = now_us();
      const int64_t f0 = thread_faults();
      load_reads(bams, iv.chrom, wb, we, opt, slab, reads[0]);
      if (opt.somatic) load_reads(normal_bams, iv.chrom, wb, we, opt, slab, reads[1]);
      const uint64_t tp = now_us();
      st.decode_seconds += (tp - td) / 1e6;
      ++st.decode_passes;
      st.inflate_gpu_chunks += std::exchange(tl_inflate_gpu, 0);
      st.inflate_host_chunks += std::exchange(tl_inflate_host, 0);
      const int64_t f1 = thread_faults();
      st.faults[0] += f1 - f0;
      pu = Pileup();
      pu.wb = wb;
      pu.depth = HugeArray<int>((size_t)(we - wb));  // zero-filled
      pu.events = HugeArray<int>((size_t)(we - wb));
      if (opt.gvcf && !opt.somatic) pu.gl = HugeArray<double>(3 * (size_t)(we - wb));
      build_pileup(seq, reads[0], opt.min_base_quality, pu);
      // activity: the sample's evidence, or in Mutect2 mode the tumor's alone
      // (Mutect2's activity profile is a tumor-evidence test; over tumor +
      // normal depth a somatic allele at the tumor's fraction reads as half
      // of it and its site is missed)
      std::vector<int64_t> sites;
      const double frac = opt.somatic ? opt.somatic_active_fraction : opt.active_fraction;
      for (int64_t p = wb; p < we; ++p) {
        const int ev = pu.events[p - wb], dp = std::max(1, pu.depth[p - wb]);
        if (ev >= 2 && ev >= frac * dp) sites.push_back(p);
      }
      if (opt.somatic) build_pileup(seq, reads[1], opt.min_base_quality, pu);
      finish_support(pu);
      clusters.clear();
      bool grow_l = false, grow_r = false;
      for (size_t i = 0; i < sites.size();) {
        size_t j = i;
        while (j + 1 < sites.size() && sites[j + 1] <= sites[j] + opt.padding) ++j;
        const int64_t first = sites[i], last = sites[j];
        i = j + 1;
        if (last < own_beg || first >= own_end) continue;  // no site in this shard's range
        if (wb > 0 && first < wb + 2 * opt.padding) grow_l = true;
        if (we < L && last + 2 * opt.padding >= we) grow_r = true;
        clusters.emplace_back(first, last);
      }
      st.pileup_seconds += (now_us() - tp) / 1e6;
      st.faults[1] += thread_faults() - f1;
      if (!grow_l && !grow_r) break;
      if (grow_l) ext_l *= 2;
      if (grow_r) ext_r *= 2;
    }
    st.reads += (int64_t)(reads[0].size() + reads[1].size());
    int64_t max_span[2] = {0, 0};
    for (int s = 0; s < 2; ++s)
      for (const Read& rd : reads[s]) max_span[s] = std::max<int64_t>(max_span[s], rd.end - rd.pos);
    const uint64_t tr = now_us();
    const int64_t fr = thread_faults();
    const double in_flush0 = st.phmm_seconds + st.genotype_seconds + st.helped_seconds;
    const int64_t hf0 = helped_faults;
    for (const auto& [first, last] : clusters) {
      for (int64_t rb = std::max<int64_t>(0, first - opt.padding); rb < std::min<int64_t>(L, last + opt.padding + 1);
           rb += opt.max_region) {
        auto g = std::make_unique<Region>();
        g->beg = rb;
        g->end = std::min<int64_t>({L, last + opt.padding + 1, rb + opt.max_region});
        // candidates: supported by >= 2 reads and a fraction of the depth
        std::vector<std::pair<int, Allele>> cs;
        const Allele key{g->beg, "", ""};
        for (auto it = std::lower_bound(pu.support.begin(), pu.support.end(), key,
                                        [](const std::pair<Allele, int>& e, const Allele& k) { return e.first < k; });
             it != pu.support.end() && it->first.pos < g->end; ++it) {
          const int dp = std::max(1, pu.depth[it->first.pos - wb]);
          if (it->first.ref_end() > g->end) continue;
          if (it->second >= 2 && it->second >= (opt.somatic ? 0.05 : 0.1) * dp) cs.emplace_back(it->second, it->first);
        }
        if (cs.empty()) continue;
        std::stable_sort(cs.begin(), cs.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
        if ((int)cs.size() > kMaxCandidates) cs.resize(kMaxCandidates);
        // a region none of whose candidates lies in the own range can produce no
        // call here (the neighbouring shard computes it)
        if (std::none_of(cs.begin(), cs.end(),
                         [&](const auto& c) { return c.second.pos >= own_beg && c.second.pos < own_end; }))
          continue;
        for (auto& c : cs) g->cands.push_back(c.second);
        std::sort(g->cands.begin(), g->cands.end());
        build_haplotypes(seq, *g);
        // reads clipped to the window, GATK-prepared, deterministic downsampling
        for (int s = 0; s < (opt.somatic ? 2 : 1); ++s) {
          // reads are in position order: start at the first that can reach beg
          // (pos >= beg - the window's longest reference span), stop at end
          std::vector<const Read*> ov;
          const HugeVec<Read>& rs = reads[s];
          auto it = std::lower_bound(rs.begin(), rs.end(), g->beg - max_span[s],
                                     [](const Read& rd, int64_t x) { return rd.pos < x; });
          for (; it != rs.end() && it->pos < g->end; ++it)
            if (it->end > g->beg) ov.push_back(&*it);
          const size_t cap = (size_t)opt.max_reads_per_region;
          const double stride = ov.size() > cap ? (double)ov.size() / cap : 1.0;
          for (double x = 0; (size_t)x < ov.size() && g->reads[s].size() < cap; x += stride) {
            const Read& rd = *ov[(size_t)x];
            size_t qs, qe;
            if (!clip_to_window(rd, g->beg, g->end, qs, qe) || qe - qs < 20) continue;
            const size_t n = qe - qs;
            if ((!rd.bi.empty() && rd.bi.size() != rd.seq.size()) || (!rd.bd.empty() && rd.bd.size() != rd.seq.size()))
              throw invalidParam("BI/BD tag length differs from the read length");
            gatk_prepare_read(rd.seq.data() + qs, rd.qual.p + qs, rd.bi.empty() ? nullptr : rd.bi.data() + qs,
                              rd.bd.empty() ? nullptr : rd.bd.data() + qs, n, rd.mapq, g->reads[s].add((int32_t)n),
                              opt.base_quality_threshold, (PcrIndelModel)opt.pcr_indel_model);
          }
        }
        if (g->reads[0].empty()) continue;
        ++st.regions;
        pending.push_back(std::move(g));
        own.emplace_back(own_beg, own_end, iv.chrom);
        if ((int)pending.size() >= opt.batch_regions) flush();
      }
    }
    st.region_seconds +=
        (now_us() - tr) / 1e6 - (st.phmm_seconds + st.genotype_seconds + st.helped_seconds - in_flush0);
    flush();
    st.faults[2] += thread_faults() - fr - (helped_faults - hf0);
    if (opt.gvcf && !opt.somatic) {
      const uint64_t tv = now_us();
      const int64_t fv = thread_faults();
      emit_gvcf(pu, own_beg, own_end, ci, calls, c0, blocks, gout);
      st.output_seconds += (now_us() - tv) / 1e6;
      st.faults[3] += thread_faults() - fv;
    }
  }
  flush();
  if (dump) std::fclose(dump);
  const uint64_t tw = now_us();
  const int64_t fw = thread_faults();
  st.calls = (int64_t)calls.size();
  // (contig index, position) order, ties in emission order: keys computed once
  // per record (the contig lookup is a name scan), then one key sort
  if (opt.gvcf && !opt.somatic) {
    HugeVec<std::pair<std::pair<int, int64_t>, uint32_t>> order;
    order.reserve(gout.size());
    for (size_t i = 0; i < gout.size(); ++i) order.emplace_back() = {{gout[i].contig, gout[i].pos}, (uint32_t)i};
    std::sort(order.begin(), order.end());
    std::string text;
    text.reserve(1u << 21);
    for (const auto& o : order) {
      const OutEntry& e = gout[o.second];
      if (e.block >= 0) {
        const GvcfBlock& k = blocks[e.block];
        const Contig& c = ref.contigs[e.contig];
        append_block_line(c.name, c.seq[k.b], k, text);
      } else {
        calls[e.call].append_line(text);
      }
      if (text.size() >= (1u << 20)) {
        out.write_text(text);
        text.clear();
      }
    }
    out.write_text(text);
  } else {
    std::vector<VcfRecord>& recs = calls;
    std::vector<std::pair<std::pair<int, int64_t>, uint32_t>> order(recs.size());
    {
      const std::string* last = nullptr;
      int last_i = -1;
      for (size_t i = 0; i < recs.size(); ++i) {
        if (!last || recs[i].chrom != *last) last = &recs[i].chrom, last_i = ref.index(recs[i].chrom);
        order[i] = {{last_i, recs[i].pos}, (uint32_t)i};
      }
    }
    std::sort(order.begin(), order.end());
    for (const auto& o : order) out.write(recs[o.second]);
  }
  st.output_seconds += (now_us() - tw) / 1e6;
  st.faults[3] += thread_faults() - fw;
  st.seconds = (now_us() - t0) / 1e6 - st.helped_seconds;
  st.cpu_seconds = thread_cpu() - cpu0 - st.helped_cpu_seconds;
  return st;
}

VcfHeader caller_vcf_header(const Reference& ref, const std::vector<std::string>& samples, bool somatic,
                            const std::string& ref_path, bool gvcf) {
  VcfHeader h;
  for (const Contig& c : ref.contigs) h.contigs.emplace_back(c.name, (int64_t)c.seq.size());
  h.samples = samples;
  h.reference = ref_path;
  h.source = somatic ? "fcs-genome mutect2 (GPU PairHMM)" : "fcs-genome htc (GPU PairHMM)";
  if (somatic) {
    h.meta = {"##INFO=<ID=TLOD,Number=1,Type=Float,Description=\"Log10 likelihood ratio of the variant in the tumor\">",
              "##INFO=<ID=NLOD,Number=1,Type=Float,Description=\"Log10 likelihood ratio of the normal being reference\">",
              "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">",
              "##FORMAT=<ID=AD,Number=R,Type=Integer,Description=\"Allelic depths (informative reads)\">",
              "##FORMAT=<ID=AF,Number=A,Type=Float,Description=\"Allele fraction\">",
              "##FILTER=<ID=PASS,Description=\"All filters passed\">"};
  } else {
    h.meta = {"##INFO=<ID=DP,Number=1,Type=Integer,Description=\"Reads in the active region\">",
              "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">",
              "##FORMAT=<ID=AD,Number=R,Type=Integer,Description=\"Allelic depths (informative reads)\">",
              "##FORMAT=<ID=DP,Number=1,Type=Integer,Description=\"Read depth\">",
              "##FORMAT=<ID=GQ,Number=1,Type=Integer,Description=\"Genotype quality\">",
              "##FORMAT=<ID=PL,Number=G,Type=Integer,Description=\"Phred-scaled genotype likelihoods\">",
              "##FILTER=<ID=PASS,Description=\"All filters passed\">"};
    if (gvcf) {
      h.meta.push_back("##ALT=<ID=NON_REF,Description=\"Represents any possible alternative allele at this location\">");
      h.meta.push_back("##INFO=<ID=END,Number=1,Type=Integer,Description=\"Stop position of the interval\">");
      h.meta.push_back(
          "##FORMAT=<ID=MIN_DP,Number=1,Type=Integer,Description=\"Minimum DP observed within the GVCF block\">");
      int lo = 0;
      for (int hi : {1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22,
                     23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44,
                     45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 70, 80, 90, 99, 100}) {
        h.meta.push_back("##GVCFBlock" + std::to_string(lo) + "-" + std::to_string(hi) + "=minGQ=" + std::to_string(lo) +
                         "(inclusive),maxGQ=" + std::to_string(hi) + "(exclusive)");
        lo = hi;
      }
    }
  }
  return h;
}

}  // namespace fcsg
