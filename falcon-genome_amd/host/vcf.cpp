#include "vcf.h"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

#include "bam.h"
#include "bgzf.h"
#include "common.h"

namespace fcsg {

void VcfRecord::append_line(std::string& s) const {
  char b[32];
  s += chrom;
  s += '\t';
  s.append(b, std::to_chars(b, b + sizeof b, pos).ptr);
  s += '\t';
  s += id;
  s += '\t';
  s += ref;
  s += '\t';
  if (alts.empty()) s += '.';
  for (size_t i = 0; i < alts.size(); ++i) {
    if (i) s += ',';
    s += alts[i];
  }
  s += '\t';
  if (qual < 0) {
    s += '.';
  } else {
    const int n = std::snprintf(b, sizeof b, "%.2f", qual);
    s.append(b, (size_t)std::max(0, std::min<int>(n, (int)sizeof b - 1)));
  }
  s += '\t';
  s += filter;
  s += '\t';
  s += info;
  if (!format.empty()) {
    s += '\t';
    s += format;
    for (const std::string& x : samples) {
      s += '\t';
      s += x;
    }
  }
  s += '\n';
}

std::string VcfRecord::to_line() const {
  std::string s;
  append_line(s);
  return s;
}

std::string VcfHeader::to_text() const {
  std::ostringstream ss;
  ss << "##fileformat=VCFv4.2\n";
  ss << "##source=" << source << '\n';
  if (!reference.empty()) ss << "##reference=file://" << reference << '\n';
  for (const std::string& m : meta) ss << m << '\n';
  for (const auto& c : contigs) ss << "##contig=<ID=" << c.first << ",length=" << c.second << ">\n";
  ss << "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO";
  if (!samples.empty()) {
    ss << "\tFORMAT";
    for (const std::string& s : samples) ss << '\t' << s;
  }
  ss << '\n';
  return ss.str();
}

struct VcfWriter::Impl {
  std::ofstream out;
  std::string buf;  // lines gathered here and written 1 MiB at a time
};

VcfWriter::VcfWriter(const std::string& path, const VcfHeader& h) : impl_(new Impl) {
  impl_->out.open(path);
  if (!impl_->out) throw fileNotFound(path + " (cannot write)");
  impl_->out << h.to_text();
}

VcfWriter::~VcfWriter() {
  try {
    close();
  } catch (...) {
  }
  delete impl_;
}

void VcfWriter::write(const VcfRecord& r) {
  r.append_line(impl_->buf);
  if (impl_->buf.size() >= (1u << 20)) {
    impl_->out.write(impl_->buf.data(), (std::streamsize)impl_->buf.size());
    impl_->buf.clear();
  }
}

void VcfWriter::write_text(const std::string& lines) {
  if (!impl_->buf.empty()) {
    impl_->out.write(impl_->buf.data(), (std::streamsize)impl_->buf.size());
    impl_->buf.clear();
  }
  impl_->out.write(lines.data(), (std::streamsize)lines.size());
}

void VcfWriter::close() {
  if (!impl_->out.is_open()) return;
  impl_->out.write(impl_->buf.data(), (std::streamsize)impl_->buf.size());
  impl_->buf.clear();
  impl_->out.close();
  if (impl_->out.fail()) throw internalError("[E::vcf] write failed");
}

void vcf_concat(const std::vector<std::string>& inputs, const std::string& output) {
  // whole parts at a time: every line of the first part, the others without
  // their '#' lines; a last line without '\n' gets one
  std::FILE* out = std::fopen(output.c_str(), "wb");
  if (!out) throw fileNotFound(output + " (cannot write)");
  std::vector<char> buf;
  std::string tail;
  for (size_t i = 0; i < inputs.size(); ++i) {
    std::FILE* in = std::fopen(inputs[i].c_str(), "rb");
    if (!in) {
      std::fclose(out);
      throw fileNotFound(inputs[i]);
    }
    std::fseek(in, 0, SEEK_END);
    const long n = std::ftell(in);
    std::fseek(in, 0, SEEK_SET);
    buf.resize((size_t)std::max(n, 0L));
    const size_t got = n > 0 ? std::fread(buf.data(), 1, (size_t)n, in) : 0;
    std::fclose(in);
    buf.resize(got);
    size_t p = 0, run = 0;  // copy [run, p) in one write when a skipped line or the end comes
    bool ok = true;
    while (p < buf.size()) {
      const char* nl = static_cast<const char*>(std::memchr(buf.data() + p, '\n', buf.size() - p));
      const size_t e = nl ? (size_t)(nl - buf.data()) + 1 : buf.size();
      if (i > 0 && buf[p] == '#') {
        ok = ok && std::fwrite(buf.data() + run, 1, p - run, out) == p - run;
        run = e;
      }
      p = e;
    }
    ok = ok && std::fwrite(buf.data() + run, 1, buf.size() - run, out) == buf.size() - run;
    if (ok && run < buf.size() && buf.back() != '\n') ok = std::fputc('\n', out) != EOF;
    if (!ok) {
      std::fclose(out);
      throw internalError("[E::vcf] write to " + output + " failed");
    }
  }
  if (std::fclose(out) != 0) throw internalError("[E::vcf] write to " + output + " failed");
}

void bgzip_file(const std::string& input, const std::string& output) {
  std::ifstream in(input, std::ios::binary);
  if (!in) throw fileNotFound(input);
  BgzfWriter w(output);
  std::vector<char> buf(1 << 20);
  while (in) {
    in.read(buf.data(), (std::streamsize)buf.size());
    const std::streamsize n = in.gcount();
    if (n > 0) w.write(buf.data(), (size_t)n);
  }
  w.close();
}

namespace {

template <typename T>
void put(std::string& s, T v) {
  s.append(reinterpret_cast<const char*>(&v), sizeof v);
}

// The index key of one VCF line (htslib's VCF preset, tbx_parse1): POS and
// the 0-based exclusive end, which INFO's END= (a GVCF <NON_REF> block, a
// symbolic allele) extends beyond POS; the field is "END=" at the start of
// INFO or the first ";END=".  False for header and empty lines.
bool vcf_index_key(const char* line, size_t len, const std::string& label, size_t& clen, int64_t& pos, int64_t& end) {
  if (len == 0 || line[0] == '#') return false;
  const char* e = line + len;
  const char* t[4];
  const char* p = line;
  for (int k = 0; k < 4; ++k) {
    t[k] = static_cast<const char*>(std::memchr(p, '\t', (size_t)(e - p)));
    if (!t[k]) throw formatError(label + ": malformed VCF line");
    p = t[k] + 1;
  }
  const auto pr = std::from_chars(t[0] + 1, t[1], pos);
  if (pr.ec != std::errc() || pr.ptr != t[1]) throw formatError(label + ": malformed VCF POS");
  const int64_t rlen = (int64_t)(t[3] - t[2] - 1);
  int64_t info_end = -1;
  const char* q = p;  // ALT
  for (int k = 0; k < 3 && q; ++k) {  // -> QUAL -> FILTER -> INFO
    q = static_cast<const char*>(std::memchr(q, '\t', (size_t)(e - q)));
    if (q) ++q;
  }
  if (q && q < e) {
    const char* ie = static_cast<const char*>(std::memchr(q, '\t', (size_t)(e - q)));
    if (!ie) ie = e;
    const char* at = nullptr;
    if (ie - q >= 4 && std::memcmp(q, "END=", 4) == 0) {
      at = q + 4;
    } else {
      for (const char* s = q; s < ie && (s = static_cast<const char*>(std::memchr(s, ';', (size_t)(ie - s)))); ++s)
        if (ie - s >= 5 && std::memcmp(s, ";END=", 5) == 0) {
          at = s + 5;
          break;
        }
    }
    if (at && at < ie && *at != '.') {
      int64_t v = 0;
      if (std::from_chars(at, ie, v).ec == std::errc()) info_end = v;
    }
  }
  clen = (size_t)(t[0] - line);
  const int64_t beg = pos - 1;
  end = info_end > beg ? info_end : beg + std::max<int64_t>(rlen, 1);
  return true;
}

// The tabix index (VCF preset) of a coordinate-sorted VCF, fed one record
// at a time with the virtual offsets of its line's start and of the next line.
class TabixBuilder {
 public:
  explicit TabixBuilder(std::string label) : label_(std::move(label)) {}
  void add(const char* line, size_t len, uint64_t beg_off, uint64_t end_off) {
    size_t clen;
    int64_t pos, end;
    if (vcf_index_key(line, len, label_, clen, pos, end)) insert(line, clen, pos, end, beg_off, end_off);
  }
  // a parsed record: chromosome name chrom[0, clen), POS, 0-based exclusive end
  void insert(const char* chrom, size_t clen, int64_t pos, int64_t end, uint64_t beg_off, uint64_t end_off) {
    int tid;
    if (!names_.empty() && names_.back().size() == clen && std::memcmp(names_.back().data(), chrom, clen) == 0) {
      tid = (int)names_.size() - 1;
    } else {
      const std::string name(chrom, clen);
      if (name_id_.count(name)) throw formatError(label_ + ": chromosome blocks not contiguous (unsorted VCF)");
      tid = (int)names_.size();
      name_id_[name] = tid;
      names_.push_back(name);
      idx_.emplace_back();
    }
    if (tid == last_tid_ && pos < last_pos_) throw formatError(label_ + ": positions not sorted");
    last_tid_ = tid;
    last_pos_ = pos;
    const int64_t beg = pos - 1;
    RefIndex& ri = idx_[tid];
    const uint32_t bin = (uint32_t)reg2bin(beg, end);
    if (tid != cache_tid_ || bin != cache_bin_) {  // records mostly repeat the previous bin
      cache_tid_ = tid;
      cache_bin_ = bin;
      cache_chunks_ = &ri.bins[bin];
    }
    auto& chunks = *cache_chunks_;
    if (!chunks.empty() && chunks.back().second == beg_off) chunks.back().second = end_off;  // extend the run
    else chunks.emplace_back(beg_off, end_off);
    const int64_t w0 = beg >> 14, w1 = (end - 1) >> 14;
    if ((int64_t)ri.linear.size() <= w1) ri.linear.resize(w1 + 1, 0);
    for (int64_t w = w0; w <= w1; ++w)
      if (ri.linear[w] == 0) ri.linear[w] = beg_off;
  }
  void write(const std::string& path) {
    std::string s = "TBI\1";
    put<int32_t>(s, (int32_t)names_.size());
    put<int32_t>(s, 2);    // format: VCF
    put<int32_t>(s, 1);    // col_seq
    put<int32_t>(s, 2);    // col_beg
    put<int32_t>(s, 0);    // col_end
    put<int32_t>(s, '#');  // meta char
    put<int32_t>(s, 0);    // skip
    std::string nm;
    for (const std::string& n : names_) nm += n + '\0';
    put<int32_t>(s, (int32_t)nm.size());
    s += nm;
    for (RefIndex& ri : idx_) {
      put<int32_t>(s, (int32_t)ri.bins.size());
      for (const auto& b : ri.bins) {
        put<uint32_t>(s, b.first);
        put<int32_t>(s, (int32_t)b.second.size());
        for (const auto& c : b.second) {
          put<uint64_t>(s, c.first);
          put<uint64_t>(s, c.second);
        }
      }
      // empty windows take the next non-empty offset to their left (tabix convention)
      for (size_t w = 1; w < ri.linear.size(); ++w)
        if (ri.linear[w] == 0) ri.linear[w] = ri.linear[w - 1];
      put<int32_t>(s, (int32_t)ri.linear.size());
      for (uint64_t o : ri.linear) put<uint64_t>(s, o);
    }
    BgzfWriter w(path);
    w.write(s);
    w.close();
  }

 private:
  struct RefIndex {
    std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
    std::vector<uint64_t> linear;  // 16 kb windows
  };
  std::string label_;
  std::vector<std::string> names_;
  std::map<std::string, int> name_id_;
  std::vector<RefIndex> idx_;
  int last_tid_ = -1;
  int64_t last_pos_ = -1;
  int cache_tid_ = -1;
  uint32_t cache_bin_ = 0;
  std::vector<std::pair<uint64_t, uint64_t>>* cache_chunks_ = nullptr;  // map values do not move
};

}  // namespace

void tabix_index_vcf(const std::string& vcf_gz) {
  BgzfReader rd(vcf_gz);
  TabixBuilder tb(vcf_gz);
  std::string line;
  for (;;) {
    const uint64_t beg_off = rd.tell();
    if (!rd.getline(line)) break;
    tb.add(line.data(), line.size(), beg_off, rd.tell());
  }
  tb.write(vcf_gz + ".tbi");
}

namespace {

// The bgzipped copy of a VCF and its tabix index in one pass over the text:
// whole-line pieces go to the BGZF writer (blocks compress on the host pool)
// and to a pool job that parses their records' index keys by uncompressed
// offset; finish() closes the writer — the blocks' compressed starts are then
// known — and enters the keys in file order with the virtual offsets a
// BgzfReader's tell() reports.
class BgzipIndexer {
 public:
  explicit BgzipIndexer(std::string gz) : gz_(std::move(gz)), w_(gz_) {}
  // lines [a, b) of *buf (b ends a line, or the data); parsed in pieces of
  // about kPiece bytes so one large part still spreads over the pool
  void add(std::shared_ptr<const std::vector<char>> buf, size_t a, size_t b) {
    if (b <= a) return;
    w_.write(buf->data() + a, b - a);
    constexpr size_t kPiece = 4u << 20;
    for (size_t p = a; p < b;) {
      size_t q = b;
      if (b - p > kPiece) {
        const void* nl = std::memchr(buf->data() + p + kPiece, '\n', b - p - kPiece);
        if (nl) q = (size_t)(static_cast<const char*>(nl) - buf->data()) + 1;
      }
      parse(buf, p, q, u_ + (p - a));
      p = q;
    }
    u_ += b - a;
  }
  void finish() {
    w_.close();
    uint64_t file_size = 0;
    if (std::FILE* f = std::fopen(gz_.c_str(), "rb")) {
      std::fseek(f, 0, SEEK_END);
      file_size = (uint64_t)std::ftell(f);
      std::fclose(f);
    }
    auto voff = [&](uint64_t x) -> uint64_t {
      // a last line without '\n': a reader's getline runs on through the EOF
      // block, so tell() is the end of the file
      return x == UINT64_MAX ? file_size << 16 : w_.voffset(x);
    };
    TabixBuilder tb(gz_);
    for (auto& job : jobs_) {
      const Parsed P = job.get();
      for (const Key& k : P.keys) {
        const std::string& c = P.names[k.chrom];
        tb.insert(c.data(), c.size(), k.pos, k.end, voff(k.u0), voff(k.u1));
      }
    }
    jobs_.clear();
    tb.write(gz_ + ".tbi");
  }

 private:
  // index keys of the lines [a, b) of *buf; `base` = uncompressed offset of a
  void parse(std::shared_ptr<const std::vector<char>> buf, size_t a, size_t b, uint64_t base) {
    jobs_.push_back(host_pool_async([buf, a, b, base, label = gz_] {
      Parsed P;
      const char* d = buf->data();
      for (size_t p = a; p < b;) {
        const char* nl = static_cast<const char*>(std::memchr(d + p, '\n', b - p));
        const size_t e = nl ? (size_t)(nl - d) : b;
        size_t clen;
        int64_t pos, end;
        if (vcf_index_key(d + p, e - p, label, clen, pos, end)) {
          if (P.names.empty() || P.names.back().size() != clen || std::memcmp(P.names.back().data(), d + p, clen) != 0)
            P.names.emplace_back(d + p, clen);
          P.keys.push_back({pos, end, base + (p - a), nl ? base + (e + 1 - a) : UINT64_MAX, (uint32_t)P.names.size() - 1});
        }
        p = e + 1;
      }
      return P;
    }));
  }

  struct Key {
    int64_t pos, end;
    uint64_t u0, u1;  // line start / next line's start (UINT64_MAX: a last line without '\n')
    uint32_t chrom;   // into Parsed::names
  };
  struct Parsed {
    std::vector<std::string> names;
    std::vector<Key> keys;
  };
  std::string gz_;
  BgzfWriter w_;
  std::vector<std::future<Parsed>> jobs_;
  uint64_t u_ = 0;  // uncompressed bytes added
};

}  // namespace

void bgzip_tabix_file(const std::string& input, const std::string& output) {
  std::FILE* in = std::fopen(input.c_str(), "rb");
  if (!in) throw fileNotFound(input);
  BgzipIndexer bx(output);
  constexpr size_t kChunk = 8u << 20;
  std::vector<char> carry;
  for (;;) {
    auto chunk = std::make_shared<std::vector<char>>(std::move(carry));
    carry = std::vector<char>();
    const size_t have = chunk->size();
    chunk->resize(have + kChunk);
    const size_t n = std::fread(chunk->data() + have, 1, kChunk, in);
    chunk->resize(have + n);
    const bool eof = n == 0;
    if (chunk->empty()) break;
    size_t cut = chunk->size();
    if (!eof) {  // whole lines only; the rest starts the next chunk
      const void* nl = memrchr(chunk->data(), '\n', chunk->size());
      cut = nl ? (size_t)(static_cast<const char*>(nl) - chunk->data()) + 1 : 0;
      carry.assign(chunk->begin() + (std::ptrdiff_t)cut, chunk->end());
      chunk->resize(cut);
      if (cut == 0) continue;
    }
    bx.add(chunk, 0, cut);
    if (eof) break;
  }
  std::fclose(in);
  bx.finish();
}

void vcf_concat_bgzip_tabix(const std::vector<std::string>& inputs, const std::string& plain, const std::string& gz,
                            bool consume_inputs) {
  // vcf_concat's text (every line of the first part, the others without
  // their '#' lines, a last line without '\n' gets one) written to `plain`
  // and, in the same pass, bgzipped + indexed as bgzip_tabix_file(plain, gz)
  const int fd = ::open(plain.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw fileNotFound(plain + " (cannot write)");
  // the plain text is written by pool jobs at known offsets (pwrite) while
  // this thread feeds the compressor; the fd closes only after every write
  // job has ended, whatever is thrown
  struct PlainOut {
    int fd;
    std::vector<std::future<bool>> writes;
    ~PlainOut() {
      for (auto& w : writes)
        if (w.valid()) w.wait();
      ::close(fd);
    }
  } po{fd, {}};
  BgzipIndexer bx(gz);
  // the next part loads on the pool while this one is written
  auto load = [](const std::string& path) {
    return host_pool_async([path] {
      std::FILE* in = std::fopen(path.c_str(), "rb");
      if (!in) throw fileNotFound(path);
      std::fseek(in, 0, SEEK_END);
      const long n = std::ftell(in);
      std::fseek(in, 0, SEEK_SET);
      auto buf = std::make_shared<std::vector<char>>((size_t)std::max(n, 0L) + 1);
      const size_t got = n > 0 ? std::fread(buf->data(), 1, (size_t)n, in) : 0;
      std::fclose(in);
      buf->resize(got);
      return buf;
    });
  };
  uint64_t off = 0;
  auto emit = [&](const std::shared_ptr<std::vector<char>>& buf, size_t a, size_t b) {
    if (b <= a) return;
    po.writes.push_back(host_pool_async([buf, a, b, fd, at = off] {
      for (size_t k = a; k < b;) {
        const ssize_t w = ::pwrite(fd, buf->data() + k, b - k, (off_t)(at + (k - a)));
        if (w <= 0) return false;
        k += (size_t)w;
      }
      return true;
    }));
    off += b - a;
    bx.add(buf, a, b);
  };
  std::future<std::shared_ptr<std::vector<char>>> next;
  if (!inputs.empty()) next = load(inputs[0]);
  for (size_t i = 0; i < inputs.size(); ++i) {
    std::shared_ptr<std::vector<char>> buf = next.get();
    if (i + 1 < inputs.size()) next = load(inputs[i + 1]);
    if (!buf->empty() && buf->back() != '\n') buf->push_back('\n');
    size_t p = 0, run = 0;  // emit [run, p) when a skipped line or the end comes
    const char* d = buf->data();
    while (p < buf->size()) {
      const char* nl = static_cast<const char*>(std::memchr(d + p, '\n', buf->size() - p));
      const size_t e = (size_t)(nl - d) + 1;
      if (i > 0 && d[p] == '#') {
        emit(buf, run, p);
        run = e;
      }
      p = e;
    }
    emit(buf, run, buf->size());
  }
  bool ok = true;
  for (auto& w : po.writes) ok = w.get() && ok;
  if (!ok) throw internalError("[E::vcf] write to " + plain + " failed");
  bx.finish();
  // the parts go only once the VCF, its .gz and .tbi are complete (a failed
  // concat leaves them for a rerun of this stage alone); removed on the pool,
  // so their page-cache pages are released in parallel
  if (consume_inputs) {
    std::vector<std::future<int>> rm;
    for (const std::string& path : inputs) rm.push_back(host_pool_async([path] { return std::remove(path.c_str()); }));
    for (auto& r : rm) r.wait();
  }
}

}  // namespace fcsg
