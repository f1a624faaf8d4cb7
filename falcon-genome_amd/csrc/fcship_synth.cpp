// Seeded synthetic workloads for the benchmark configurations of BASELINE.json
// (C2: PairHMM pairs, C3: bwa-mem seed-extension tasks), as specified in
// SURVEY.md §8(d).  Every pair / read draws from its own counter-based stream
// (splitmix64 of seed and index), so the output is independent of threading.
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "fcship_internal.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed, uint64_t stream) : s(seed * 0x9E3779B97F4A7C15ull ^ (stream + 0x632BE59BD9B4E019ull)) {
    next();
    next();
  }
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  // uniform in [0, n)
  uint64_t below(uint64_t n) { return n ? next() % n : 0; }
  double unit() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

const char kBase[4] = {'A', 'C', 'G', 'T'};

template <typename F>
void parallel_for(int64_t n, F&& f) {
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < 4096) nt = 1;
  std::vector<std::thread> th;
  const int64_t chunk = (n + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const int64_t lo = t * chunk, hi = std::min<int64_t>(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back([&f, lo, hi] {
      for (int64_t i = lo; i < hi; ++i) f(i);
    });
  }
  for (auto& x : th) x.join();
}

int32_t hap_len_of(uint64_t seed, int64_t p, int32_t hmin, int32_t hmax) {
  Rng r(seed, (uint64_t)p * 2 + 1);
  return hmin + (int32_t)r.below((uint64_t)(hmax - hmin + 1));
}

}  // namespace

extern "C" {

int fcs_synth_phmm_sizes(uint64_t seed, int64_t n_pairs, int32_t R, int32_t hmin, int32_t hmax, int64_t* read_bytes,
                         int64_t* hap_bytes) {
  if (n_pairs < 0 || R <= 0 || hmin <= 0 || hmax < hmin || !read_bytes || !hap_bytes)
    return fcs::fail(FCS_ERR_INVALID, "[E::fcs_synth_phmm_sizes] bad arguments");
  int64_t hb = 0;
  for (int64_t p = 0; p < n_pairs; ++p) hb += hap_len_of(seed, p, hmin, hmax);
  *read_bytes = n_pairs * (int64_t)R;
  *hap_bytes = hb;
  return FCS_OK;
}

int fcs_synth_phmm(uint64_t seed, int64_t n_pairs, int32_t R, int32_t hmin, int32_t hmax, uint8_t* read_bases,
                   uint8_t* read_bq, uint8_t* read_iq, uint8_t* read_dq, uint8_t* read_gcp, int64_t* read_off,
                   int32_t* read_len, uint8_t* hap_bases, int64_t* hap_off, int32_t* hap_len) {
  if (n_pairs < 0 || R <= 0 || hmin <= 0 || hmax < hmin)
    return fcs::fail(FCS_ERR_INVALID, "[E::fcs_synth_phmm] bad arguments");
  int64_t off = 0;
  for (int64_t p = 0; p < n_pairs; ++p) {
    hap_len[p] = hap_len_of(seed, p, hmin, hmax);
    hap_off[p] = off;
    off += hap_len[p];
    read_off[p] = p * (int64_t)R;
  }
  parallel_for(n_pairs, [&](int64_t p) {
    Rng r(seed, (uint64_t)p * 2);
    const int32_t H = hap_len[p];
    uint8_t* h = hap_bases + hap_off[p];
    for (int32_t c = 0; c < H; ++c) h[c] = kBase[r.below(4)];
    uint8_t* rb = read_bases + read_off[p];
    uint8_t* bq = read_bq + read_off[p];
    int32_t start = H > R ? (int32_t)r.below((uint64_t)(H - R + 1)) : 0;
    int32_t n = 0, c = start;
    while (n < R && c < H) {
      const double u = r.unit();
      if (u < 0.0005) {  // 0.1% indels, half insertions
        const int len = 1 + (int)r.below(3);
        for (int k = 0; k < len && n < R; ++k) rb[n++] = kBase[r.below(4)];
        continue;
      }
      if (u < 0.001) {
        c += 1 + (int)r.below(3);
        continue;
      }
      uint8_t b = h[c++];
      if (r.unit() < 0.01) {  // 1% substitutions
        uint8_t nb;
        do nb = kBase[r.below(4)]; while (nb == b);
        b = nb;
      }
      rb[n++] = b;
    }
    read_len[p] = n;
    for (int32_t k = 0; k < R; ++k) {
      bq[k] = (uint8_t)(10 + r.below(31));
      read_iq[read_off[p] + k] = 45;
      read_dq[read_off[p] + k] = 45;
      read_gcp[read_off[p] + k] = 10;
      if (k >= n) rb[k] = 'A';
    }
  });
  return FCS_OK;
}

namespace {

// Mutated copy of ref[pos..) of length L (codes 0..3): 0.5% substitutions,
// 0.05% indels.  Returns the number of reference bases consumed.
int64_t mutate_read(Rng& r, const uint8_t* ref, int64_t ref_len, int64_t pos, int32_t L, uint8_t* out) {
  int32_t n = 0;
  int64_t c = pos;
  while (n < L && c < ref_len) {
    const double u = r.unit();
    if (u < 0.00025) {
      out[n++] = (uint8_t)r.below(4);
      continue;
    }
    if (u < 0.0005) {
      ++c;
      continue;
    }
    uint8_t b = ref[c++];
    if (r.unit() < 0.005) b = (uint8_t)((b + 1 + r.below(3)) & 3);
    out[n++] = b;
  }
  while (n < L) out[n++] = (uint8_t)r.below(4);
  return c - pos;
}

struct BswPlan {
  int64_t n_tasks = 0, qbytes = 0, tbytes = 0;
};

// Walks the generator once; if the output pointers are non-null, fills them.
int synth_bsw_impl(uint64_t seed, int64_t n_reads, int32_t L, int64_t ref_len, int32_t w, int32_t mode,
                   int32_t fq, int32_t ft, uint8_t* qbuf, int64_t* qoff, int32_t* qlen, uint8_t* tbuf, int64_t* toff,
                   int32_t* tlen, int32_t* h0, int32_t* wv, BswPlan* plan) {
  std::vector<uint8_t> ref((size_t)ref_len);
  {
    Rng r(seed, 0xFEEDull);
    for (int64_t i = 0; i < ref_len; ++i) ref[i] = (uint8_t)r.below(4);
  }
  std::vector<uint8_t> rd((size_t)std::max(L, fq) + 8);
  int64_t nt = 0, qo = 0, to = 0;
  auto emit = [&](const uint8_t* q, int32_t ql, const uint8_t* t, int32_t tl, int32_t hz, bool rev) {
    if (qbuf) {
      qoff[nt] = qo;
      toff[nt] = to;
      qlen[nt] = ql;
      tlen[nt] = tl;
      h0[nt] = hz;
      wv[nt] = w;
      for (int32_t k = 0; k < ql; ++k) qbuf[qo + k] = rev ? q[ql - 1 - k] : q[k];
      for (int32_t k = 0; k < tl; ++k) tbuf[to + k] = rev ? t[tl - 1 - k] : t[k];
    }
    ++nt;
    qo += ql;
    to += tl;
  };
  for (int64_t rdi = 0; rdi < n_reads; ++rdi) {
    Rng r(seed, (uint64_t)rdi + 0x100000000ull);
    if (mode == 1) {
      const int64_t pos = (int64_t)r.below((uint64_t)std::max<int64_t>(1, ref_len - ft));
      mutate_read(r, ref.data(), ref_len, pos, fq, rd.data());
      const int32_t tl = (int32_t)std::min<int64_t>(ft, ref_len - pos);
      emit(rd.data(), fq, ref.data() + pos, tl, 30, false);
      continue;
    }
    const int64_t pos = (int64_t)r.below((uint64_t)std::max<int64_t>(1, ref_len - 2 * L));
    mutate_read(r, ref.data(), ref_len, pos, L, rd.data());
    const int32_t slen = 19 + (int32_t)r.below(22);  // seed length 19..40
    const int32_t qbeg = (int32_t)r.below((uint64_t)(L - slen + 1));
    const int32_t qend = qbeg + slen;
    const int64_t rbeg = pos + qbeg;  // seed start on the reference
    if (qbeg > 0) {                   // left extension: reversed query prefix vs reversed reference
      const int64_t avail = rbeg;
      const int32_t tl = (int32_t)std::min<int64_t>(qbeg + w, avail);
      emit(rd.data(), qbeg, ref.data() + (rbeg - tl), tl, slen, true);
    }
    if (qend < L) {  // right extension
      const int32_t ql = L - qend;
      const int64_t rs = rbeg + slen;
      const int64_t avail = ref_len - rs;
      const int32_t tl = (int32_t)std::min<int64_t>(ql + w, avail);
      emit(rd.data() + qend, ql, ref.data() + rs, tl, slen + qbeg, false);
    }
  }
  if (plan) {
    plan->n_tasks = nt;
    plan->qbytes = qo;
    plan->tbytes = to;
  }
  return FCS_OK;
}

}  // namespace

int fcs_synth_bsw_sizes(uint64_t seed, int64_t n_reads, int32_t read_len, int64_t ref_len, int32_t w, int32_t mode,
                        int32_t fixed_q, int32_t fixed_t, int64_t* n_tasks, int64_t* qbytes, int64_t* tbytes) {
  if (n_reads < 0 || read_len < 41 || ref_len < 4 * (int64_t)read_len + 4 * (int64_t)w || w < 0 ||
      (mode == 1 && (fixed_q <= 0 || fixed_t <= 0 || fixed_t >= ref_len)) || !n_tasks || !qbytes || !tbytes)
    return fcs::fail(FCS_ERR_INVALID, "[E::fcs_synth_bsw_sizes] bad arguments");
  BswPlan pl;
  synth_bsw_impl(seed, n_reads, read_len, ref_len, w, mode, fixed_q, fixed_t, nullptr, nullptr, nullptr, nullptr,
                 nullptr, nullptr, nullptr, nullptr, &pl);
  *n_tasks = pl.n_tasks;
  *qbytes = pl.qbytes;
  *tbytes = pl.tbytes;
  return FCS_OK;
}

int fcs_synth_bsw(uint64_t seed, int64_t n_reads, int32_t read_len, int64_t ref_len, int32_t w, int32_t mode,
                  int32_t fixed_q, int32_t fixed_t, uint8_t* qbuf, int64_t* qoff, int32_t* qlen, uint8_t* tbuf,
                  int64_t* toff, int32_t* tlen, int32_t* h0, int32_t* wv, int64_t* n_tasks) {
  if (!qbuf || !qoff || !qlen || !tbuf || !toff || !tlen || !h0 || !wv || !n_tasks)
    return fcs::fail(FCS_ERR_INVALID, "[E::fcs_synth_bsw] null buffer");
  BswPlan pl;
  int rc = synth_bsw_impl(seed, n_reads, read_len, ref_len, w, mode, fixed_q, fixed_t, qbuf, qoff, qlen, tbuf, toff,
                          tlen, h0, wv, &pl);
  *n_tasks = pl.n_tasks;
  return rc;
}

}  // extern "C"
