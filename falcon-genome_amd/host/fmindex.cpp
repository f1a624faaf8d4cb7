#include "fmindex.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstring>
#include <stdexcept>

#include "common.h"

namespace fcsg {

namespace {

template <typename I>
constexpr I kEmpty = ~I(0);

template <typename C>
void buckets(const C* s, int64_t n, int64_t K, std::vector<int64_t>& bkt, bool end) {
  std::fill(bkt.begin(), bkt.end(), 0);
  for (int64_t i = 0; i < n; ++i) ++bkt[s[i]];
  int64_t sum = 0;
  for (int64_t c = 0; c < K; ++c) {
    sum += bkt[c];
    bkt[c] = end ? sum : sum - bkt[c];
  }
}

template <typename C, typename I>
void induce(const C* s, I* sa, int64_t n, int64_t K, const std::vector<uint8_t>& t, std::vector<int64_t>& bkt) {
  buckets(s, n, K, bkt, false);  // L-type suffixes, left to right from bucket starts
  for (int64_t i = 0; i < n; ++i) {
    if (sa[i] == kEmpty<I> || sa[i] == 0) continue;
    const int64_t j = (int64_t)sa[i] - 1;
    if (!t[j]) sa[bkt[s[j]]++] = (I)j;
  }
  buckets(s, n, K, bkt, true);  // S-type suffixes, right to left from bucket ends
  for (int64_t i = n - 1; i >= 0; --i) {
    if (sa[i] == kEmpty<I> || sa[i] == 0) continue;
    const int64_t j = (int64_t)sa[i] - 1;
    if (t[j]) sa[--bkt[s[j]]] = (I)j;
  }
}

// SA-IS (Nong, Zhang and Chan 2009): sort the LMS substrings by induction,
// name them, recurse on the reduced string (stored in the SA's upper half)
// when names repeat, then induce the full order from the sorted LMS suffixes.
template <typename C, typename I>
void sais_t(const C* s, I* sa, int64_t n, int64_t K) {
  std::vector<uint8_t> t(n);  // 1 = S-type
  t[n - 1] = 1;
  for (int64_t i = n - 2; i >= 0; --i) t[i] = s[i] < s[i + 1] || (s[i] == s[i + 1] && t[i + 1]);
  auto lms = [&](int64_t i) { return i > 0 && t[i] && !t[i - 1]; };
  std::vector<int64_t> bkt(K);
  std::fill(sa, sa + n, kEmpty<I>);
  buckets(s, n, K, bkt, true);
  for (int64_t i = 1; i < n; ++i)
    if (lms(i)) sa[--bkt[s[i]]] = (I)i;
  induce(s, sa, n, K, t, bkt);
  int64_t n1 = 0;
  for (int64_t i = 0; i < n; ++i)
    if (sa[i] != kEmpty<I> && lms((int64_t)sa[i])) sa[n1++] = sa[i];
  std::fill(sa + n1, sa + n, kEmpty<I>);
  int64_t name = 0, prev = -1;
  for (int64_t i = 0; i < n1; ++i) {
    const int64_t pos = (int64_t)sa[i];
    bool diff = false;
    for (int64_t d = 0; d < n; ++d) {
      if (prev == -1 || s[pos + d] != s[prev + d] || t[pos + d] != t[prev + d]) {
        diff = true;
        break;
      }
      if (d > 0 && (lms(pos + d) || lms(prev + d))) break;
    }
    if (diff) {
      ++name;
      prev = pos;
    }
    sa[n1 + pos / 2] = (I)(name - 1);
  }
  for (int64_t i = n - 1, j = n - 1; i >= n1; --i)
    if (sa[i] != kEmpty<I>) sa[j--] = sa[i];
  I* s1 = sa + n - n1;
  if (name < n1) {
    sais_t<I, I>(s1, sa, n1, name);
  } else {
    for (int64_t i = 0; i < n1; ++i) sa[s1[i]] = (I)i;
  }
  for (int64_t i = 1, j = 0; i < n; ++i)
    if (lms(i)) s1[j++] = (I)i;
  for (int64_t i = 0; i < n1; ++i) sa[i] = s1[sa[i]];
  std::fill(sa + n1, sa + n, kEmpty<I>);
  buckets(s, n, K, bkt, true);
  for (int64_t i = n1 - 1; i >= 0; --i) {
    const I j = sa[i];
    sa[i] = kEmpty<I>;
    sa[--bkt[s[j]]] = j;
  }
  induce(s, sa, n, K, t, bkt);
}

}  // namespace

void sais(const uint8_t* s, uint64_t* sa, int64_t n, int K) { sais_t<uint8_t, uint64_t>(s, sa, n, K); }

FmdIndex::FmdIndex(const std::vector<std::vector<uint8_t>>& contigs, int sa_intv) {
  // F = 5 C_1 5 C_2 ... 5 C_n 5;  T = F revcomp(F) $
  std::vector<uint8_t> T;
  int64_t total = 1;
  for (const auto& c : contigs) total += (int64_t)c.size() + 1;
  T.reserve(2 * total + 1);
  for (const auto& c : contigs) {
    T.push_back(5);
    cstart_.push_back((int64_t)T.size());
    clen_.push_back((int64_t)c.size());
    for (uint8_t b : c) T.push_back(b < 4 ? (uint8_t)(b + 1) : (uint8_t)5);
  }
  T.push_back(5);
  flen_ = (int64_t)T.size();
  for (int64_t i = flen_ - 1; i >= 0; --i) T.push_back(T[i] == 5 ? (uint8_t)5 : (uint8_t)(5 - T[i]));
  T.push_back(0);
  n_ = (int64_t)T.size();
  digest_ = text_digest(contigs);
  std::vector<uint64_t> sa(n_);
  sais(T.data(), sa.data(), n_, 6);
  C_.assign(7, 0);
  for (uint8_t c : T) ++C_[c + 1];
  for (int c = 1; c < 7; ++c) C_[c] += C_[c - 1];
  const int64_t nb = (n_ + 63) / 64;
  occ_store_.assign(8 * (size_t)(nb + 1) + 8, 0);
  uint64_t* occ = occ_store_.data();
  while (reinterpret_cast<uintptr_t>(occ) & 63) ++occ;
  occ_ = occ;
  nocc_ = 8 * (nb + 1);
  uint64_t run[4] = {0, 0, 0, 0};
  for (int64_t b = 0; b <= nb; ++b) {
    uint64_t* B = occ + 8 * b;
    for (int c = 0; c < 4; ++c) B[c] = run[c];
    for (int64_t i = 64 * b; i < std::min(n_, 64 * b + 64); ++i) {
      const uint64_t p = sa[i];
      const uint32_t ch = p ? T[p - 1] : 0;  // BWT symbol
      if (ch >= 1 && ch <= 4) {
        B[4 + ch - 1] |= 1ull << (i & 63);
        ++run[ch - 1];
      } else {
        special_store_.emplace_back(i, (int64_t)p);  // no LF step from this row
      }
    }
  }
  if (sa_intv <= 0) {
    sa_intv = 1;
    while ((uint64_t)n_ / sa_intv * 8 > (8ull << 30)) sa_intv *= 2;
  }
  intv_ = sa_intv;
  if (intv_ == 1) {
    sa_store_ = std::move(sa);
    special_store_.clear();
  } else {
    sa_store_.resize((size_t)((n_ + intv_ - 1) / intv_));
    for (size_t k = 0; k < sa_store_.size(); ++k) sa_store_[k] = sa[k * intv_];
    std::vector<std::pair<int64_t, int64_t>> sp;  // sampled rows need no special entry
    for (const auto& e : special_store_)
      if (e.first % intv_ != 0) sp.push_back(e);
    special_store_.swap(sp);
  }
  sa_ = sa_store_.data();
  nsa_ = (int64_t)sa_store_.size();
  special_ = special_store_.data();
  nspecial_ = (int64_t)special_store_.size();
}

FmdIndex::~FmdIndex() {
  if (map_) ::munmap(map_, map_len_);
}

// A digest of the whole reference text (every contig's length and every base
// code, eight codes per mixing step): a saved index is used only for the exact
// text it was built from.  An edit that keeps the lengths (IUPAC -> N, a
// masked or patched base) changes it.
uint64_t FmdIndex::text_digest(const std::vector<std::vector<uint8_t>>& contigs) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t v) {
    h ^= v;
    h *= 1099511628211ull;
    h ^= h >> 29;
  };
  for (const auto& c : contigs) {
    mix(c.size());
    const size_t n8 = c.size() / 8;
    for (size_t i = 0; i < n8; ++i) {
      uint64_t w;
      std::memcpy(&w, c.data() + 8 * i, 8);
      mix(w);
    }
    uint64_t tail = 0;
    for (size_t i = 8 * n8; i < c.size(); ++i) tail = tail << 8 | c[i];
    mix(tail);
  }
  return h;
}

namespace {
constexpr char kFmdMagic[8] = {'F', 'C', 'S', 'F', 'M', 'D', '0', '2'};  // 02: whole-text digest
struct FmdHeader {
  char magic[8];
  int64_t n, flen, intv, ncontig, nocc, nsa, nspecial;
  uint64_t digest;
  int64_t C[7];
};
size_t align64(size_t x) { return (x + 63) & ~(size_t)63; }
}  // namespace

void FmdIndex::save(const std::string& path) const {
  FmdHeader h{};
  std::memcpy(h.magic, kFmdMagic, 8);
  h.n = n_;
  h.flen = flen_;
  h.intv = intv_;
  h.ncontig = (int64_t)cstart_.size();
  h.nocc = nocc_;
  h.nsa = nsa_;
  h.nspecial = nspecial_;
  h.digest = digest_;
  for (int c = 0; c < 7; ++c) h.C[c] = C_[c];
  const std::string tmp = path + ".tmp";
  std::FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) throw fileNotFound(tmp + " (cannot open for writing)");
  size_t off = 0;
  auto put = [&](const void* p, size_t n) {
    if (n && std::fwrite(p, 1, n, f) != n) {
      std::fclose(f);
      throw internalError("[E::fcsg] cannot write " + tmp);
    }
    off += n;
  };
  auto pad = [&] {
    static const char z[64] = {0};
    put(z, align64(off) - off);
  };
  put(&h, sizeof h);
  put(cstart_.data(), 8 * cstart_.size());
  put(clen_.data(), 8 * clen_.size());
  pad();
  put(occ_, 8 * (size_t)nocc_);
  pad();
  put(sa_, 8 * (size_t)nsa_);
  pad();
  put(special_, 16 * (size_t)nspecial_);
  if (std::fclose(f) != 0) throw internalError("[E::fcsg] cannot write " + tmp);
  if (std::rename(tmp.c_str(), path.c_str()) != 0) throw internalError("[E::fcsg] cannot rename " + tmp);
}

std::unique_ptr<FmdIndex> FmdIndex::load(const std::string& path, const std::vector<std::vector<uint8_t>>& contigs) {
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (::fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(FmdHeader)) {
    ::close(fd);
    return nullptr;
  }
  void* m = ::mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  ::close(fd);
  if (m == MAP_FAILED) return nullptr;
  std::unique_ptr<FmdIndex> ix(new FmdIndex());
  ix->map_ = m;
  ix->map_len_ = (size_t)st.st_size;
  const char* base = static_cast<const char*>(m);
  FmdHeader h;
  std::memcpy(&h, base, sizeof h);
  if (std::memcmp(h.magic, kFmdMagic, 8) != 0 || h.ncontig != (int64_t)contigs.size() || h.intv < 1 ||
      h.digest != text_digest(contigs))
    return nullptr;
  size_t off = sizeof h;
  ix->cstart_.assign(reinterpret_cast<const int64_t*>(base + off), reinterpret_cast<const int64_t*>(base + off) + h.ncontig);
  off += 8 * (size_t)h.ncontig;
  ix->clen_.assign(reinterpret_cast<const int64_t*>(base + off), reinterpret_cast<const int64_t*>(base + off) + h.ncontig);
  off = align64(off + 8 * (size_t)h.ncontig);
  int64_t total = 1;
  for (int64_t c = 0; c < h.ncontig; ++c) {
    if (ix->clen_[c] != (int64_t)contigs[c].size()) return nullptr;
    total += ix->clen_[c] + 1;
  }
  // the header's sizes must be the ones this text gives (the constructor's
  // layout), so that no lookup can leave the mapped arrays
  const int64_t n = 2 * total + 1;
  if (h.flen != total || h.n != n || h.nocc != 8 * ((n + 63) / 64 + 1) || h.nsa != (n + h.intv - 1) / h.intv ||
      h.nspecial < 0 || h.nspecial > n || h.C[0] != 0 || h.C[6] != n)
    return nullptr;
  for (int c = 1; c < 7; ++c)
    if (h.C[c] < h.C[c - 1]) return nullptr;
  const size_t need = align64(align64(off + 8 * (size_t)h.nocc) + 8 * (size_t)h.nsa) + 16 * (size_t)h.nspecial;
  if (need > ix->map_len_) return nullptr;
  ix->n_ = h.n;
  ix->flen_ = h.flen;
  ix->intv_ = (int)h.intv;
  ix->digest_ = h.digest;
  ix->C_.assign(h.C, h.C + 7);
  ix->occ_ = reinterpret_cast<const uint64_t*>(base + off);
  ix->nocc_ = h.nocc;
  off = align64(off + 8 * (size_t)h.nocc);
  ix->sa_ = reinterpret_cast<const uint64_t*>(base + off);
  ix->nsa_ = h.nsa;
  off = align64(off + 8 * (size_t)h.nsa);
  ix->special_ = reinterpret_cast<const std::pair<int64_t, int64_t>*>(base + off);
  ix->nspecial_ = h.nspecial;
  return ix;
}

int64_t FmdIndex::sa_at(int64_t row) const {
  // SA[LF(i)] = SA[i] - 1: walk back to a sampled row (bwa bwt_sa)
  int64_t steps = 0;
  for (;;) {
    if (row % intv_ == 0) return (int64_t)sa_[row / intv_] + steps;
    const uint64_t* B = occ_ + 8 * (row >> 6);
    const uint64_t bit = 1ull << (row & 63);
    int c = -1;
    for (int k = 0; k < 4; ++k)
      if (B[4 + k] & bit) c = k;
    if (c < 0) {  // $ or a separator precedes this suffix: stored
      const auto* e = std::lower_bound(special_, special_ + nspecial_, std::make_pair(row, (int64_t)INT64_MIN));
      if (e == special_ + nspecial_ || e->first != row) throw internalError("[E::fcsg] FMD-index special row missing");
      return e->second + steps;
    }
    row = C_[c + 1] + (int64_t)(B[c] + (uint64_t)__builtin_popcountll(B[4 + c] & (bit - 1)));
    ++steps;
  }
}

void FmdIndex::occ4(int64_t i, int64_t o[4]) const {
  if (i <= 0) {
    o[0] = o[1] = o[2] = o[3] = 0;
    return;
  }
  const uint64_t* B = occ_ + 8 * (i >> 6);  // i <= n: at most the totals block
  const uint64_t m = (1ull << (i & 63)) - 1;
  for (int c = 0; c < 4; ++c) o[c] = (int64_t)(B[c] + (uint64_t)__builtin_popcountll(B[4 + c] & m));
}

void FmdIndex::set_intv(int c, BiInterval& iv) const {
  iv.k = C_[c];
  iv.s = C_[c + 1] - C_[c];
  iv.l = C_[5 - c];
}

// bwa bwt_extend: the four one-base extensions of ik, backward (cP, is_back)
// or forward (P comp(c), reported at index c: the backward extension of
// revcomp(P) by c).  The other coordinate follows from the counts: the
// revcomp(P) x (resp. P x) suffixes are ordered by x, and x = $ never occurs
// (the base before $ is a separator).
void FmdIndex::extend(const BiInterval& ik, BiInterval ok[5], bool is_back) const {
  const int64_t base = is_back ? ik.k : ik.l;
  int64_t tk[4], tl[4];
  occ4(base, tk);
  occ4(base + ik.s, tl);
  for (int c = 1; c <= 4; ++c) {
    (is_back ? ok[c].k : ok[c].l) = C_[c] + tk[c - 1];
    ok[c].s = tl[c - 1] - tk[c - 1];
  }
  int64_t o = is_back ? ik.l : ik.k;
  for (int c = 4; c >= 1; --c) {
    (is_back ? ok[c].l : ok[c].k) = o;
    o += ok[c].s;
  }
}

int FmdIndex::smem1(const uint8_t* q, int len, int x, int64_t min_intv, std::vector<BiInterval>& mem) const {
  mem.clear();
  if (q[x] > 3) return x + 1;
  if (min_intv < 1) min_intv = 1;
  thread_local std::vector<BiInterval> a0, a1;  // reused: one smem1 call per query position
  a0.clear();
  a1.clear();
  std::vector<BiInterval>*prev = &a0, *curr = &a1;
  BiInterval ik, ok[5];
  set_intv(q[x] + 1, ik);
  ik.qe = x + 1;
  int i;
  for (i = x + 1; i < len; ++i) {  // forward search
    if (ik.s < min_intv) break;
    if (q[i] < 4) {
      const int c = 4 - q[i];  // index of the forward extension by q[i]
      extend(ik, ok, false);
      if (ok[c].s != ik.s) {
        curr->push_back(ik);
        if (ok[c].s < min_intv) break;
      }
      ik = ok[c];
      ik.qe = i + 1;
    } else {
      curr->push_back(ik);
      break;
    }
  }
  if (i == len) curr->push_back(ik);
  std::reverse(curr->begin(), curr->end());  // longest forward match first
  const int ret = curr->front().qe;
  std::swap(curr, prev);
  for (i = x - 1; i >= -1; --i) {  // backward search for MEMs
    const int c = i < 0 ? -1 : q[i] < 4 ? q[i] + 1 : -1;
    curr->clear();
    for (const BiInterval& p : *prev) {
      if (c >= 0 && ik.s >= min_intv) extend(p, ok, true);  // bwa tests ik, not p
      if (c < 0 || ok[c].s < min_intv) {
        if (curr->empty()) {  // no longer match in this round: p is maximal
          if (mem.empty() || i + 1 < mem.back().qb) {
            ik = p;
            ik.qb = i + 1;
            mem.push_back(ik);
          }
        }
      } else if (curr->empty() || ok[c].s != curr->back().s) {
        ok[c].qe = p.qe;
        curr->push_back(ok[c]);
      }
    }
    if (curr->empty()) break;
    std::swap(curr, prev);
  }
  std::reverse(mem.begin(), mem.end());  // by start coordinate
  return ret;
}

void FmdIndex::collect(const uint8_t* q, int len, int min_len, int split_len, int split_width, int64_t max_mem_intv,
                       std::vector<BiInterval>& out) const {
  out.clear();
  std::vector<BiInterval> m;
  for (int x = 0; x < len;) {
    if (q[x] < 4) {
      x = smem1(q, len, x, 1, m);
      for (const BiInterval& p : m)
        if (p.qe - p.qb >= min_len) out.push_back(p);
    } else {
      ++x;
    }
  }
  const size_t n0 = out.size();
  for (size_t k = 0; k < n0; ++k) {  // re-seeding inside long SMEMs with few hits
    const BiInterval p = out[k];
    if (p.qe - p.qb < split_len || p.s > split_width) continue;
    smem1(q, len, (p.qb + p.qe) >> 1, p.s + 1, m);
    for (const BiInterval& r : m)
      if (r.qe - r.qb >= min_len) out.push_back(r);
  }
  if (max_mem_intv > 0) {  // third round (bwt_seed_strategy1): the first forward match of
    // length >= min_len from each x with fewer than max_mem_intv occurrences
    for (int x = 0; x < len;) {
      if (q[x] > 3) {
        ++x;
        continue;
      }
      BiInterval ik, ok[5];
      set_intv(q[x] + 1, ik);
      int next = len;
      for (int i = x + 1; i < len; ++i) {
        if (q[i] > 3) {
          next = i + 1;
          break;
        }
        extend(ik, ok, false);
        const BiInterval& o = ok[4 - q[i]];
        if (o.s < max_mem_intv && i - x >= min_len) {
          if (o.s > 0) {
            BiInterval m = o;
            m.qb = x;
            m.qe = i + 1;
            out.push_back(m);
          }
          next = i + 1;
          break;
        }
        ik = o;
      }
      x = next;
    }
  }
  std::stable_sort(out.begin(), out.end(), [](const BiInterval& a, const BiInterval& b) {
    return a.qb != b.qb ? a.qb < b.qb : a.qe < b.qe;
  });
}

void FmdIndex::locate(const BiInterval& iv, int64_t j, int& contig, int64_t& off, bool& rev) const {
  int64_t p = sa_at(iv.k + j);
  const int64_t len = iv.qe - iv.qb;
  rev = p >= flen_;
  if (rev) p = 2 * flen_ - p - len;  // start of the reverse-strand match on F
  const auto it = std::upper_bound(cstart_.begin(), cstart_.end(), p);
  contig = (int)(it - cstart_.begin()) - 1;
  off = p - cstart_[contig];
}

}  // namespace fcsg
