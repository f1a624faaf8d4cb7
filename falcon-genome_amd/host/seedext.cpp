#include "seedext.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <string>

#include "common.h"

namespace fcsg {

int bwa_cal_max_gap(const fcs_bsw_params& p, int qlen, int w) {
  const int a = p.mat[0];
  const int l_del = (int)((double)(qlen * a - p.o_del) / p.e_del + 1.);
  const int l_ins = (int)((double)(qlen * a - p.o_ins) / p.e_ins + 1.);
  int l = std::max(l_del, l_ins);
  l = std::max(l, 1);
  return std::min(l, w << 1);
}

int bwa_infer_bw(int l1, int l2, int score, int a, int q, int r) {
  if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;  // equal lengths need at least two gaps
  int w = (int)((double)(std::min(l1, l2) * a - score - q) / r + 2.);
  if (w < std::abs(l1 - l2)) w = std::abs(l1 - l2);
  return w;
}

int bwa_cigar_band(const fcs_bsw_params& p, int l, int64_t rlen, int w_) {
  const int a = p.mat[0];
  const int max_ins = (int)((double)(((l + 1) >> 1) * a - p.o_ins) / p.e_ins + 1.);
  const int max_del = (int)((double)(((l + 1) >> 1) * a - p.o_del) / p.e_del + 1.);
  int max_gap = std::max(std::max(max_ins, max_del), 1);
  const int diff = std::abs((int)rlen - l);
  int w = (max_gap + diff + 1) >> 1;
  w = std::min(w, w_);
  return std::max(w, diff + 3);
}

namespace {

struct Side {
  std::vector<uint8_t> q, t;  // reversed for the left extension
  int h0 = 0, w = 0;
  bool run = false;
};

// One round of ksw_extend2 tasks on the GPU.
void run_extend(std::vector<fcs_bsw_task>& tasks, const fcs_bsw_params& p, int gpu, std::vector<fcs_bsw_result>& res,
                SeedExtStats& st) {
  res.resize(tasks.size());
  if (tasks.empty()) return;
  const uint64_t g0 = now_us();
  if (fcs_bsw_extend(tasks.data(), (int32_t)tasks.size(), &p, res.data(), gpu) != FCS_OK)
    throw failedCommand(std::string(fcs_last_error()));
  st.gpu_seconds += (now_us() - g0) / 1e6;
  st.ext_tasks += (int64_t)tasks.size();
}

// The extension rounds of one side for every job that needs it: try w, then 2w
// where the score changed and max_off >= 3/4 w (MAX_BAND_TRY = 2).  `prev` is
// bwa's a->score before each try.
void extend_side(std::vector<Side>& sides, std::vector<int>& prev, const fcs_bsw_params& p, int w0, int gpu,
                 std::vector<fcs_bsw_result>& last, SeedExtStats& st) {
  std::vector<int> todo;
  for (size_t i = 0; i < sides.size(); ++i)
    if (sides[i].run) todo.push_back((int)i);
  last.assign(sides.size(), fcs_bsw_result{});
  for (int pass = 0; pass < 2 && !todo.empty(); ++pass) {
    std::vector<fcs_bsw_task> tasks;
    for (int i : todo) {
      Side& s = sides[i];
      s.w = w0 << pass;
      tasks.push_back({(int32_t)s.q.size(), (int32_t)s.t.size(), s.h0, s.w, s.q.data(), s.t.data()});
    }
    std::vector<fcs_bsw_result> res;
    run_extend(tasks, p, gpu, res, st);
    std::vector<int> again;
    for (size_t k = 0; k < todo.size(); ++k) {
      const int i = todo[k];
      const fcs_bsw_result& x = res[k];
      last[i] = x;
      const int w = sides[i].w;
      const bool stop = x.score == prev[i] || x.max_off < (w >> 1) + (w >> 2);
      prev[i] = x.score;
      if (!stop && pass + 1 < 2) again.push_back(i);
    }
    todo.swap(again);
  }
}

}  // namespace

void extend_seeds(const std::vector<SeedJob>& jobs, const fcs_bsw_params& p_in, const SeedExtOptions& opt,
                  std::vector<SeedAln>& out, SeedExtStats& st) {
  const size_t n = jobs.size();
  out.assign(n, SeedAln{});
  const int a = p_in.mat[0];
  fcs_bsw_params pl = p_in, pr = p_in;
  pl.end_bonus = opt.pen_clip5;
  pr.end_bonus = opt.pen_clip3;
  std::vector<int64_t> rmax0(n), rmax1(n);
  std::vector<Side> left(n), right(n);
  std::vector<int> prev(n, -1), aw0(n, opt.w), aw1(n, opt.w);
  for (size_t i = 0; i < n; ++i) {
    const SeedJob& J = jobs[i];
    if (J.seed_len <= 0 || J.seed_q < 0 || J.seed_q + J.seed_len > J.qlen || J.seed_r < 0 ||
        J.seed_r + J.seed_len > J.rlen)
      throw invalidParam("extend_seeds: seed outside its query or contig");
  }
  parallel_for(n, opt.threads, [&](size_t i) {
    const SeedJob& J = jobs[i];
    const int rest = J.qlen - J.seed_q - J.seed_len;
    if (J.win_lo >= 0 || J.win_hi >= 0) {  // the chain's window (bwa's rmax over all its seeds)
      rmax0[i] = std::max<int64_t>(0, J.win_lo);
      rmax1[i] = std::min<int64_t>(J.rlen, J.win_hi);
      if (rmax0[i] > J.seed_r || rmax1[i] < J.seed_r + J.seed_len)
        throw invalidParam("extend_seeds: chain window does not contain the seed");
    } else {
      rmax0[i] = std::max<int64_t>(0, J.seed_r - (J.seed_q + bwa_cal_max_gap(p_in, J.seed_q, opt.w)));
      rmax1[i] = std::min<int64_t>(J.rlen, J.seed_r + J.seed_len + rest + bwa_cal_max_gap(p_in, rest, opt.w));
    }
    SeedAln& A = out[i];
    if (J.seed_q > 0) {
      Side& s = left[i];
      s.run = true;
      s.q.resize(J.seed_q);
      for (int k = 0; k < J.seed_q; ++k) s.q[k] = J.q[J.seed_q - 1 - k];
      const int64_t tmp = J.seed_r - rmax0[i];
      s.t.resize(tmp);
      for (int64_t k = 0; k < tmp; ++k) s.t[k] = J.ref[J.seed_r - 1 - k];
      s.h0 = J.seed_len * a;
    } else {
      A.score = A.truesc = J.seed_len * a;
      A.qb = 0;
      A.rb = J.seed_r;
    }
  });
  std::vector<fcs_bsw_result> lres, rres;
  extend_side(left, prev, pl, opt.w, opt.gpu, lres, st);
  for (size_t i = 0; i < n; ++i) {
    if (!left[i].run) continue;
    const SeedJob& J = jobs[i];
    SeedAln& A = out[i];
    const fcs_bsw_result& x = lres[i];
    aw0[i] = left[i].w;
    A.score = x.score;
    if (x.gscore <= 0 || x.gscore <= A.score - opt.pen_clip5) {  // local extension
      A.qb = J.seed_q - x.qle;
      A.rb = J.seed_r - x.tle;
      A.truesc = A.score;
    } else {  // to-end extension
      A.qb = 0;
      A.rb = J.seed_r - x.gtle;
      A.truesc = x.gscore;
    }
  }
  std::vector<int> sc0(n, 0);
  parallel_for(n, opt.threads, [&](size_t i) {
    const SeedJob& J = jobs[i];
    SeedAln& A = out[i];
    const int qe = J.seed_q + J.seed_len;
    if (qe != J.qlen) {
      Side& s = right[i];
      s.run = true;
      const int64_t re = J.seed_r + J.seed_len - rmax0[i];
      s.q.assign(J.q + qe, J.q + J.qlen);
      const int64_t tl = rmax1[i] - rmax0[i] - re;
      s.t.assign(J.ref + rmax0[i] + re, J.ref + rmax0[i] + re + std::max<int64_t>(tl, 0));
      s.h0 = sc0[i] = A.score;
      prev[i] = A.score;
    } else {
      A.qe = J.qlen;
      A.re = J.seed_r + J.seed_len;
    }
  });
  extend_side(right, prev, pr, opt.w, opt.gpu, rres, st);
  for (size_t i = 0; i < n; ++i) {
    if (!right[i].run) continue;
    const SeedJob& J = jobs[i];
    SeedAln& A = out[i];
    const fcs_bsw_result& x = rres[i];
    aw1[i] = right[i].w;
    const int qe = J.seed_q + J.seed_len;
    const int64_t re = J.seed_r + J.seed_len - rmax0[i];
    A.score = x.score;
    if (x.gscore <= 0 || x.gscore <= A.score - opt.pen_clip3) {  // local extension
      A.qe = qe + x.qle;
      A.re = rmax0[i] + re + x.tle;
      A.truesc += A.score - sc0[i];
    } else {  // to-end extension
      A.qe = J.qlen;
      A.re = rmax0[i] + re + x.gtle;
      A.truesc += x.gscore - sc0[i];
    }
  }
  for (size_t i = 0; i < n; ++i) out[i].w = std::max(aw0[i], aw1[i]);
  if (opt.want_cigar) global_cigars(jobs, p_in, opt, out, st);
}

void global_cigars(const std::vector<SeedJob>& jobs, const fcs_bsw_params& p_in, const SeedExtOptions& opt,
                   std::vector<SeedAln>& out, SeedExtStats& st) {
  const size_t n = jobs.size();
  const int a = p_in.mat[0];
  // ---- mem_reg2aln: the CIGAR by banded global alignment, widened up to three times
  std::vector<int> w2(n, 0), last_sc(n, INT_MIN), tries(n, 0);
  std::vector<int> todo;
  for (size_t i = 0; i < n; ++i) {
    SeedAln& A = out[i];
    A.cigar.clear();
    if (A.qe <= A.qb || A.re <= A.rb) continue;
    const int l1 = A.qe - A.qb, l2 = (int)(A.re - A.rb);
    int w = std::max(bwa_infer_bw(l1, l2, A.truesc, a, p_in.o_del, p_in.e_del),
                     bwa_infer_bw(l1, l2, A.truesc, a, p_in.o_ins, p_in.e_ins));
    if (w > opt.w) w = std::min(w, A.w);
    w2[i] = w;
    todo.push_back((int)i);
  }
  while (!todo.empty()) {
    std::vector<fcs_bsw_task> tasks;
    std::vector<int> dp;  // jobs that go through ksw_global2 this round
    std::vector<int64_t> off;
    std::vector<int32_t> cap;
    int64_t tot = 0;
    for (int i : todo) {
      w2[i] = std::min(w2[i], opt.w << 2);
      SeedAln& A = out[i];
      const SeedJob& J = jobs[i];
      const int l = A.qe - A.qb;
      const int64_t rlen = A.re - A.rb;
      if (l == rlen && w2[i] == 0) {  // bwa_gen_cigar2: equal lengths, no band: no DP
        int sc = 0;
        for (int k = 0; k < l; ++k) sc += p_in.mat[J.q[A.qb + k] * 5 + J.ref[A.rb + k]];
        A.gscore = sc;
        A.gw = 0;
        A.cigar.assign(1, (uint32_t)l << 4);
        continue;
      }
      A.gw = bwa_cigar_band(p_in, l, rlen, w2[i]);
      tasks.push_back({(int32_t)l, (int32_t)rlen, 0, A.gw, J.q + A.qb, J.ref + A.rb});
      dp.push_back(i);
      off.push_back(tot);
      cap.push_back((int32_t)(l + rlen + 1));
      tot += cap.back();
    }
    if (!tasks.empty()) {
      std::vector<int32_t> scores(tasks.size()), ncig(tasks.size());
      // capacity l + rlen + 1 ops per task, mostly unused: not zero-filled
      std::unique_ptr<uint32_t[]> arena(new uint32_t[(size_t)std::max<int64_t>(tot, 1)]);
      const uint64_t g0 = now_us();
      if (fcs_bsw_global(tasks.data(), (int32_t)tasks.size(), &p_in, scores.data(), arena.get(), off.data(),
                         cap.data(), ncig.data(), opt.gpu) != FCS_OK)
        throw failedCommand(std::string(fcs_last_error()));
      st.gpu_seconds += (now_us() - g0) / 1e6;
      st.global_tasks += (int64_t)tasks.size();
      parallel_for(dp.size(), opt.threads, [&](size_t k) {
        SeedAln& A = out[dp[k]];
        A.cigar.assign(arena.get() + off[k], arena.get() + off[k] + ncig[k]);
        A.gscore = scores[k];
      });
    }
    std::vector<int> again;
    for (int i : todo) {
      SeedAln& A = out[i];
      const int sc = A.gscore;
      if (sc == last_sc[i] || w2[i] == opt.w << 2) continue;
      last_sc[i] = sc;
      w2[i] <<= 1;
      if (++tries[i] < 3 && sc < A.truesc - a) again.push_back(i);
    }
    todo.swap(again);
  }
}

void global_scores(const std::vector<GlobalScoreJob>& jobs, const fcs_bsw_params& p, int gpu, std::vector<int>& scores,
                   SeedExtStats& st) {
  scores.assign(jobs.size(), 0);
  std::vector<fcs_bsw_task> tasks;
  std::vector<size_t> who;
  for (size_t i = 0; i < jobs.size(); ++i) {
    const GlobalScoreJob& J = jobs[i];
    const int l = J.qe - J.qb;
    const int64_t rlen = J.re - J.rb;
    if (l == rlen && J.w == 0) {
      int sc = 0;
      for (int k = 0; k < l; ++k) sc += p.mat[J.q[J.qb + k] * 5 + J.ref[J.rb + k]];
      scores[i] = sc;
      continue;
    }
    tasks.push_back({(int32_t)l, (int32_t)rlen, 0, bwa_cigar_band(p, l, rlen, J.w), J.q + J.qb, J.ref + J.rb});
    who.push_back(i);
  }
  if (tasks.empty()) return;
  std::vector<int32_t> sc(tasks.size());
  const uint64_t g0 = now_us();
  if (fcs_bsw_global(tasks.data(), (int32_t)tasks.size(), &p, sc.data(), nullptr, nullptr, nullptr, nullptr, gpu) !=
      FCS_OK)
    throw failedCommand(std::string(fcs_last_error()));
  st.gpu_seconds += (now_us() - g0) / 1e6;
  st.global_tasks += (int64_t)tasks.size();
  for (size_t k = 0; k < who.size(); ++k) scores[who[k]] = sc[k];
}

}  // namespace fcsg
