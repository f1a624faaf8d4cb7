#include "bam.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#include <deque>
#include <future>
#include <map>
#include <sstream>

#include "bgzf.h"
#include "common.h"

namespace fcsg {

namespace {

const char kSeqNt16[] = "=ACMGRSVTWYHKDBN";

struct Nt16Table {
  uint8_t tab[256];
  Nt16Table() {
    for (int i = 0; i < 256; ++i) tab[i] = 15;
    for (int k = 0; k < 16; ++k) {
      tab[(uint8_t)kSeqNt16[k]] = (uint8_t)k;
      tab[(uint8_t)std::tolower(kSeqNt16[k])] = (uint8_t)k;
    }
  }
};

// Built once by a function-local static (thread-safe initialisation): the
// aligner's record builders call this from several threads.
uint8_t nt16_code(char c) {
  static const Nt16Table t;
  return t.tab[(uint8_t)c];
}

template <typename T>
void put(std::string& s, T v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof v);  // BAM is little-endian, as is x86-64
}
template <typename T>
T get(const uint8_t* p) {
  T v;
  std::memcpy(&v, p, sizeof v);
  return v;
}

// Size of one aux value of type t at p (for skipping), 0 on malformed data.
size_t aux_value_size(char t, const uint8_t* p, const uint8_t* end) {
  switch (t) {
    case 'A': case 'c': case 'C': return 1;
    case 's': case 'S': return 2;
    case 'i': case 'I': case 'f': return 4;
    case 'Z': case 'H': {
      const void* z = std::memchr(p, 0, end - p);
      return z ? (size_t)(static_cast<const uint8_t*>(z) - p) + 1 : 0;
    }
    case 'B': {
      if (end - p < 5) return 0;
      const char st = (char)p[0];
      const uint32_t n = get<uint32_t>(p + 1);
      const size_t es = (st == 'c' || st == 'C') ? 1 : (st == 's' || st == 'S') ? 2 : 4;
      return 5 + es * n;
    }
    default: return 0;
  }
}

// Offset of tag in the raw aux bytes b[0, n) (pointing at the 2 tag bytes), or npos.
size_t find_aux_raw(const uint8_t* b, size_t n, const char tag[2]) {
  const uint8_t* e = b + n;
  const uint8_t* p = b;
  while (p + 3 <= e) {
    const size_t vs = aux_value_size((char)p[2], p + 3, e);
    if (vs == 0) throw formatError("malformed BAM aux data");
    if (p[0] == (uint8_t)tag[0] && p[1] == (uint8_t)tag[1]) return (size_t)(p - b);
    p += 3 + vs;
  }
  return std::string::npos;
}

size_t find_aux(const std::string& aux, const char tag[2]) {
  return find_aux_raw(reinterpret_cast<const uint8_t*>(aux.data()), aux.size(), tag);
}

// Both bases of every packed byte (high nibble first).
struct SeqPairTable {
  char pair[256][2];
  SeqPairTable() {
    for (int b = 0; b < 256; ++b) {
      pair[b][0] = kSeqNt16[b >> 4];
      pair[b][1] = kSeqNt16[b & 0xf];
    }
  }
};

void erase_aux(std::string& aux, const char tag[2]) {
  const size_t k = find_aux(aux, tag);
  if (k == std::string::npos) return;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(aux.data()) + k;
  const size_t vs = aux_value_size((char)p[2], p + 3, reinterpret_cast<const uint8_t*>(aux.data()) + aux.size());
  aux.erase(k, 3 + vs);
}

}  // namespace

int64_t cigar_ref_len(const std::vector<uint32_t>& cigar) {
  int64_t n = 0;
  for (uint32_t c : cigar) {
    const CigarOp op = cigar_op(c);
    if (op == kM || op == kD || op == kN || op == kEq || op == kX) n += cigar_len(c);
  }
  return n;
}

std::string cigar_string(const std::vector<uint32_t>& cigar) {
  if (cigar.empty()) return "*";
  static const char ops[] = "MIDNSHP=X";
  std::string s;
  for (uint32_t c : cigar) s += std::to_string(cigar_len(c)) + ops[std::min<uint32_t>(c & 0xf, 8)];
  return s;
}

std::vector<uint32_t> parse_cigar(const std::string& s) {
  std::vector<uint32_t> out;
  if (s == "*") return out;
  static const std::string ops = "MIDNSHP=X";
  uint32_t n = 0;
  bool digit = false;
  for (char c : s) {
    if (c >= '0' && c <= '9') {
      n = n * 10 + (uint32_t)(c - '0');
      digit = true;
      continue;
    }
    const size_t k = ops.find(c);
    if (k == std::string::npos || !digit) throw formatError("bad CIGAR " + s);
    out.push_back(cigar_pack(n, (CigarOp)k));
    n = 0;
    digit = false;
  }
  if (digit) throw formatError("bad CIGAR " + s);
  return out;
}

uint16_t reg2bin(int64_t beg, int64_t end) {
  --end;
  if (beg >> 14 == end >> 14) return (uint16_t)(((1 << 15) - 1) / 7 + (beg >> 14));
  if (beg >> 17 == end >> 17) return (uint16_t)(((1 << 12) - 1) / 7 + (beg >> 17));
  if (beg >> 20 == end >> 20) return (uint16_t)(((1 << 9) - 1) / 7 + (beg >> 20));
  if (beg >> 23 == end >> 23) return (uint16_t)(((1 << 6) - 1) / 7 + (beg >> 23));
  if (beg >> 26 == end >> 26) return (uint16_t)(((1 << 3) - 1) / 7 + (beg >> 26));
  return 0;
}

bool BamRecord::get_aux_string(const char tag[2], std::string& out) const {
  return bam_aux_string(reinterpret_cast<const uint8_t*>(aux.data()), aux.size(), tag, out);
}

bool bam_aux_string(const uint8_t* aux, size_t n, const char tag[2], std::string& out) {
  const size_t k = find_aux_raw(aux, n, tag);
  if (k == std::string::npos || aux[k + 2] != 'Z') return false;
  out.assign(reinterpret_cast<const char*>(aux) + k + 3);  // NUL-terminated: find_aux_raw checked
  return true;
}

void decode_bam_seq(const uint8_t* packed, int32_t l_seq, char* out) {
  static const SeqPairTable t;
  int32_t i = 0;
  for (; i + 1 < l_seq; i += 2) std::memcpy(out + i, t.pair[packed[i / 2]], 2);
  if (i < l_seq) out[i] = t.pair[packed[i / 2]][0];
}

bool BamRecord::get_aux_int(const char tag[2], int64_t& out) const {
  const size_t k = find_aux(aux, tag);
  if (k == std::string::npos) return false;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(aux.data()) + k + 3;
  switch (aux[k + 2]) {
    case 'c': out = (int8_t)p[0]; return true;
    case 'C': out = p[0]; return true;
    case 's': out = get<int16_t>(p); return true;
    case 'S': out = get<uint16_t>(p); return true;
    case 'i': out = get<int32_t>(p); return true;
    case 'I': out = get<uint32_t>(p); return true;
    default: return false;
  }
}

void BamRecord::set_aux_string(const char tag[2], const std::string& v) {
  erase_aux(aux, tag);
  aux += tag[0];
  aux += tag[1];
  aux += 'Z';
  aux += v;
  aux += '\0';
}

void BamRecord::set_aux_int(const char tag[2], int32_t v) {
  erase_aux(aux, tag);
  aux += tag[0];
  aux += tag[1];
  aux += 'i';
  put<int32_t>(aux, v);
}

int BamHeader::ref_index(const std::string& name) const {
  for (size_t i = 0; i < names.size(); ++i)
    if (names[i] == name) return (int)i;
  return -1;
}

void encode_bam_record(const BamRecord& r, std::string& s) {
  s.clear();
  const int64_t end = r.cigar.empty() ? r.pos + 1 : r.end();
  put<int32_t>(s, r.ref_id);
  put<int32_t>(s, r.pos);
  put<uint8_t>(s, (uint8_t)(r.name.size() + 1));
  put<uint8_t>(s, r.mapq);
  put<uint16_t>(s, reg2bin(r.pos < 0 ? -1 : r.pos, r.pos < 0 ? 0 : end));
  put<uint16_t>(s, (uint16_t)r.cigar.size());
  put<uint16_t>(s, r.flag);
  put<int32_t>(s, (int32_t)r.seq.size());
  put<int32_t>(s, r.next_ref_id);
  put<int32_t>(s, r.next_pos);
  put<int32_t>(s, r.tlen);
  s += r.name;
  s += '\0';
  for (uint32_t c : r.cigar) put<uint32_t>(s, c);
  for (size_t i = 0; i < r.seq.size(); i += 2) {
    const uint8_t hi = nt16_code(r.seq[i]);
    const uint8_t lo = i + 1 < r.seq.size() ? nt16_code(r.seq[i + 1]) : 0;
    s += (char)((hi << 4) | lo);
  }
  if (r.qual.empty()) s.append(r.seq.size(), (char)0xff);
  else {
    if (r.qual.size() != r.seq.size()) throw formatError("qual length differs from seq length in " + r.name);
    s.append(reinterpret_cast<const char*>(r.qual.data()), r.qual.size());
  }
  s += r.aux;
}

void decode_bam_record(const uint8_t* p, size_t n, BamRecord& r) {
  if (n < 32) throw formatError("short BAM record");
  r.ref_id = get<int32_t>(p);
  r.pos = get<int32_t>(p + 4);
  const uint8_t l_name = p[8];
  r.mapq = p[9];
  const uint16_t n_cigar = get<uint16_t>(p + 12);
  r.flag = get<uint16_t>(p + 14);
  const int32_t l_seq = get<int32_t>(p + 16);
  r.next_ref_id = get<int32_t>(p + 20);
  r.next_pos = get<int32_t>(p + 24);
  r.tlen = get<int32_t>(p + 28);
  size_t k = 32;
  const size_t need = k + l_name + 4 * (size_t)n_cigar + (l_seq + 1) / 2 + (size_t)l_seq;
  if (l_seq < 0 || need > n) throw formatError("truncated BAM record");
  r.name.assign(reinterpret_cast<const char*>(p + k), l_name ? l_name - 1 : 0);
  k += l_name;
  r.cigar.resize(n_cigar);
  for (uint16_t i = 0; i < n_cigar; ++i) r.cigar[i] = get<uint32_t>(p + k + 4 * i);
  k += 4 * (size_t)n_cigar;
  r.seq.resize(l_seq);
  decode_bam_seq(p + k, l_seq, r.seq.data());
  k += (l_seq + 1) / 2;
  if (l_seq > 0 && p[k] == 0xff) r.qual.clear();
  else r.qual.assign(p + k, p + k + l_seq);
  k += l_seq;
  r.aux.assign(reinterpret_cast<const char*>(p + k), n - k);
}

// ------------------------------------------------------------------ files
BamWriter::BamWriter(const std::string& path, const BamHeader& h, int level)
    : path_(path), nref_(h.names.size()), bgzf_(path, level) {
  std::string s = "BAM\1";
  put<int32_t>(s, (int32_t)h.text.size());
  s += h.text;
  put<int32_t>(s, (int32_t)h.names.size());
  for (size_t i = 0; i < h.names.size(); ++i) {
    put<int32_t>(s, (int32_t)h.names[i].size() + 1);
    s += h.names[i];
    s += '\0';
    put<int32_t>(s, (int32_t)h.lengths[i]);
  }
  bgzf_.write(s);
  bgzf_.flush();  // records start on a block boundary
}

void BamWriter::write(const BamRecord& r) {
  encode_bam_record(r, rec_);
  write_encoded(r, rec_);
}

void BamWriter::write_all(const std::vector<const BamRecord*>& recs) {
  // pieces of records encoded on the host pool, written in order; the
  // uncompressed stream (and so the file and its index) is write()'s
  struct Piece {
    std::string bytes;                // [block_size][body] per record
    std::vector<int64_t> meta;        // per record: ref_id, pos, end, encoded size
  };
  constexpr size_t kPiece = 8192;
  const size_t npieces = (recs.size() + kPiece - 1) / kPiece;
  const size_t window = 4 * (size_t)host_pool_size();
  std::deque<std::future<Piece>> inflight;
  size_t next = 0;
  auto submit = [&] {
    const size_t a = next * kPiece, b = std::min(recs.size(), a + kPiece);
    ++next;
    inflight.push_back(host_pool_async([&recs, a, b, index = index_] {
      Piece pc;
      std::string body;
      if (index) pc.meta.reserve(4 * (b - a));
      for (size_t i = a; i < b; ++i) {
        const BamRecord& r = *recs[i];
        encode_bam_record(r, body);
        const int32_t bs = (int32_t)body.size();
        pc.bytes.append(reinterpret_cast<const char*>(&bs), 4);
        pc.bytes += body;
        if (index) pc.meta.insert(pc.meta.end(), {r.ref_id, r.pos, r.ref_id >= 0 ? r.end() : 0, 4 + (int64_t)bs});
      }
      return pc;
    }));
  };
  while (next < npieces && inflight.size() < window) submit();
  while (!inflight.empty()) {
    const Piece pc = inflight.front().get();
    inflight.pop_front();
    if (next < npieces) submit();
    uint64_t u = bgzf_.upos();
    bgzf_.write(pc.bytes);
    if (index_)
      for (size_t k = 0; k < pc.meta.size(); k += 4) {
        const uint64_t u1 = u + (uint64_t)pc.meta[k + 3];
        spans_.push_back({(int32_t)pc.meta[k], pc.meta[k + 1], pc.meta[k + 2], u, u1});
        u = u1;
      }
  }
}

void BamWriter::write_encoded(const BamRecord& r, const std::string& body) {
  const int32_t bs = (int32_t)body.size();
  const uint64_t u0 = bgzf_.upos();
  bgzf_.write(&bs, 4);
  bgzf_.write(body);
  if (index_) spans_.push_back({r.ref_id, r.pos, r.ref_id >= 0 ? r.end() : 0, u0, bgzf_.upos()});
}

BamReader::BamReader(const std::string& path) : bgzf_(path) {
  char magic[4];
  if (!bgzf_.read_exact(magic, 4) || std::memcmp(magic, "BAM\1", 4) != 0) throw formatError(path + " is not a BAM file");
  int32_t l_text = 0, n_ref = 0;
  bgzf_.read_exact(&l_text, 4);
  hdr_.text.resize(l_text);
  if (l_text) bgzf_.read_exact(&hdr_.text[0], l_text);
  const size_t z = hdr_.text.find('\0');
  if (z != std::string::npos) hdr_.text.resize(z);
  bgzf_.read_exact(&n_ref, 4);
  for (int32_t i = 0; i < n_ref; ++i) {
    int32_t ln = 0, lr = 0;
    bgzf_.read_exact(&ln, 4);
    std::string nm(ln, '\0');
    bgzf_.read_exact(&nm[0], ln);
    nm.resize(ln ? ln - 1 : 0);
    bgzf_.read_exact(&lr, 4);
    hdr_.names.push_back(nm);
    hdr_.lengths.push_back(lr);
  }
}

bool BamReader::next(BamRecord& r) {
  const uint8_t* body;
  size_t n;
  if (!next_raw(body, n)) return false;
  decode_bam_record(body, n, r);
  return true;
}

bool BamReader::next_raw(const uint8_t*& body, size_t& n) {
  int32_t bs = 0;
  if (const uint8_t* p = bgzf_.view(4)) std::memcpy(&bs, p, 4);
  else if (!bgzf_.read_exact(&bs, 4)) return false;
  if (bs < 32) throw formatError("bad BAM block_size");
  if (const uint8_t* p = bgzf_.view((size_t)bs)) {  // inside one block: no copy
    body = p;
    n = (size_t)bs;
    return true;
  }
  buf_.resize(bs);
  bgzf_.read_exact(buf_.data(), bs);
  body = buf_.data();
  n = buf_.size();
  return true;
}

}  // namespace fcsg

namespace fcsg {

namespace {

// The BAI of a coordinate-sorted BAM, fed record by record with the virtual
// offsets of its start and of the next record.
class BaiBuilder {
 public:
  BaiBuilder(size_t nref, std::string label) : bins_(nref), linear_(nref), label_(std::move(label)) {}
  void add(int32_t ref_id, int64_t pos, int64_t rend, uint64_t beg_off, uint64_t end_off) {
    if (ref_id < 0) {
      ++n_no_coor_;
      return;
    }
    if ((size_t)ref_id >= bins_.size()) throw formatError(label_ + ": record reference id outside the header");
    if (ref_id < last_tid_ || (ref_id == last_tid_ && pos < last_pos_))
      throw formatError(label_ + " is not coordinate-sorted; cannot index");
    last_tid_ = ref_id;
    last_pos_ = pos;
    const int64_t beg = pos, end = std::max<int64_t>(rend, beg + 1);
    auto& ch = bins_[ref_id][reg2bin(beg, end)];
    if (!ch.empty() && ch.back().second == beg_off) ch.back().second = end_off;
    else ch.emplace_back(beg_off, end_off);
    auto& lin = linear_[ref_id];
    const int64_t w1 = (end - 1) >> 14;
    if ((int64_t)lin.size() <= w1) lin.resize(w1 + 1, 0);
    for (int64_t w = beg >> 14; w <= w1; ++w)
      if (lin[w] == 0) lin[w] = beg_off;
  }
  void write(const std::string& path) {
    std::string s = "BAI\1";
    put<int32_t>(s, (int32_t)bins_.size());
    for (size_t t = 0; t < bins_.size(); ++t) {
      put<int32_t>(s, (int32_t)bins_[t].size());
      for (const auto& b : bins_[t]) {
        put<uint32_t>(s, b.first);
        put<int32_t>(s, (int32_t)b.second.size());
        for (const auto& c : b.second) {
          put<uint64_t>(s, c.first);
          put<uint64_t>(s, c.second);
        }
      }
      auto& lin = linear_[t];
      for (size_t w = 1; w < lin.size(); ++w)
        if (lin[w] == 0) lin[w] = lin[w - 1];
      put<int32_t>(s, (int32_t)lin.size());
      for (uint64_t o : lin) put<uint64_t>(s, o);
    }
    put<uint64_t>(s, n_no_coor_);
    write_file(path, s);
  }

 private:
  std::vector<std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>>> bins_;
  std::vector<std::vector<uint64_t>> linear_;
  std::string label_;
  uint64_t n_no_coor_ = 0;
  int last_tid_ = -1;
  int64_t last_pos_ = -1;
};

}  // namespace

void bam_index_build(const std::string& bam_path) {
  BamReader rd(bam_path);
  BaiBuilder bb(rd.header().names.size(), bam_path);
  BamRecord r;
  for (;;) {
    const uint64_t beg_off = rd.tell();
    if (!rd.next(r)) break;
    bb.add(r.ref_id, r.pos, r.ref_id >= 0 ? r.end() : 0, beg_off, rd.tell());
  }
  bb.write(bam_path + ".bai");
}

void BamWriter::close() {
  if (closed_) return;
  closed_ = true;
  bgzf_.close();
  if (!index_) return;
  BaiBuilder bb(nref_, path_);
  for (const Span& s : spans_) bb.add(s.ref_id, s.beg, s.end, bgzf_.voffset(s.u0), bgzf_.voffset(s.u1));
  spans_.clear();
  spans_.shrink_to_fit();
  bb.write(path_ + ".bai");
}

BamIndex::BamIndex(const std::string& bai_path) {
  const std::string d = read_file(bai_path);
  const uint8_t* p = reinterpret_cast<const uint8_t*>(d.data());
  const uint8_t* e = p + d.size();
  auto need = [&](size_t n) {
    if ((size_t)(e - p) < n) throw formatError(bai_path + ": truncated BAI");
  };
  need(8);
  if (std::memcmp(p, "BAI\1", 4) != 0) throw formatError(bai_path + " is not a BAI index");
  const int32_t nref = get<int32_t>(p + 4);
  p += 8;
  linear_.resize(nref);
  for (int32_t t = 0; t < nref; ++t) {
    need(4);
    const int32_t nbin = get<int32_t>(p);
    p += 4;
    for (int32_t b = 0; b < nbin; ++b) {
      need(8);
      const int32_t nch = get<int32_t>(p + 4);
      p += 8;
      need(16 * (size_t)nch);
      p += 16 * (size_t)nch;
    }
    need(4);
    const int32_t nint = get<int32_t>(p);
    p += 4;
    need(8 * (size_t)nint);
    linear_[t].resize(nint);
    for (int32_t k = 0; k < nint; ++k) linear_[t][k] = get<uint64_t>(p + 8 * k);
    p += 8 * (size_t)nint;
  }
}

uint64_t BamIndex::seek_offset(int tid, int64_t beg) const {
  if (tid < 0 || tid >= (int)linear_.size() || linear_[tid].empty()) return 0;
  const auto& lin = linear_[tid];
  const int64_t w = std::min<int64_t>(beg >> 14, (int64_t)lin.size() - 1);
  return lin[w];
}

}  // namespace fcsg
