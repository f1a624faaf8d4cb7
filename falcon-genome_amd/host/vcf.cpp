#include "vcf.h"

#include <algorithm>
#include <charconv>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
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

// The tabix index (VCF preset) of a coordinate-sorted VCF, fed one record
// line at a time with the virtual offsets of its start and of the next line.
class TabixBuilder {
 public:
  explicit TabixBuilder(std::string label) : label_(std::move(label)) {}
  void add(const char* line, size_t len, uint64_t beg_off, uint64_t end_off) {
    if (len == 0 || line[0] == '#') return;
    const char* e = line + len;
    const char* t[4];
    const char* p = line;
    for (int k = 0; k < 4; ++k) {
      t[k] = static_cast<const char*>(std::memchr(p, '\t', (size_t)(e - p)));
      if (!t[k]) throw formatError(label_ + ": malformed VCF line");
      p = t[k] + 1;
    }
    char* pe = nullptr;
    const int64_t pos = std::strtoll(t[0] + 1, &pe, 10);
    if (pe != t[1]) throw formatError(label_ + ": malformed VCF POS");
    const int64_t rlen = (int64_t)(t[3] - t[2] - 1);
    // htslib's VCF preset (tbx_parse1): INFO's END= (a GVCF <NON_REF> block,
    // a symbolic allele) beyond POS sets the record's end (1-based inclusive =
    // 0-based exclusive); the field is "END=" at the start of INFO or the
    // first ";END="
    int64_t info_end = -1;
    {
      const char* q = p;  // ALT
      for (int k = 0; k < 3 && q; ++k) {  // -> QUAL -> FILTER -> INFO
        q = static_cast<const char*>(std::memchr(q, '\t', (size_t)(e - q)));
        if (q) ++q;
      }
      if (q && q < e) {
        const char* ie = static_cast<const char*>(std::memchr(q, '\t', (size_t)(e - q)));
        const std::string info(q, ie ? ie : e);
        size_t at = std::string::npos;
        if (info.compare(0, 4, "END=") == 0) at = 4;
        else if (const size_t k = info.find(";END="); k != std::string::npos) at = k + 5;
        if (at != std::string::npos && at < info.size() && info[at] != '.') info_end = std::strtoll(info.c_str() + at, nullptr, 10);
      }
    }
    const size_t clen = (size_t)(t[0] - line);
    int tid;
    if (!names_.empty() && names_.back().size() == clen && std::memcmp(names_.back().data(), line, clen) == 0) {
      tid = (int)names_.size() - 1;
    } else {
      const std::string chrom(line, clen);
      if (name_id_.count(chrom)) throw formatError(label_ + ": chromosome blocks not contiguous (unsorted VCF)");
      tid = (int)names_.size();
      name_id_[chrom] = tid;
      names_.push_back(chrom);
      idx_.emplace_back();
    }
    if (tid == last_tid_ && pos < last_pos_) throw formatError(label_ + ": positions not sorted");
    last_tid_ = tid;
    last_pos_ = pos;
    const int64_t beg = pos - 1, end = info_end > beg ? info_end : beg + std::max<int64_t>(rlen, 1);
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

void bgzip_tabix_file(const std::string& input, const std::string& output) {
  // One pass over the plain VCF: its bytes go to the (parallel) BGZF writer
  // and its record lines to the index, by uncompressed offset; the writer
  // turns those into the virtual offsets a BgzfReader's tell() reports once
  // the blocks' compressed starts are known (after close).
  std::FILE* in = std::fopen(input.c_str(), "rb");
  if (!in) throw fileNotFound(input);
  BgzfWriter w(output);
  struct Rec {
    uint64_t u0, u1, at;  // line start / end offsets; `at` into `lines`
    uint32_t len;
  };
  std::vector<Rec> recs;
  std::string lines;  // the record lines' first eight columns (through INFO: enough for the index)
  std::vector<char> buf(4 << 20);
  std::string carry;
  uint64_t u = 0;  // uncompressed offset of buf[0] - carry.size()
  auto take = [&](const char* s, size_t n, uint64_t u0) {
    if (n == 0 || s[0] == '#') return false;
    size_t keep = n, tabs = 0;
    for (size_t k = 0; k < n; ++k)
      if (s[k] == '\t' && ++tabs == 8) {
        keep = k;
        break;
      }
    recs.push_back({u0, u0 + n + 1, (uint64_t)lines.size(), (uint32_t)keep});
    lines.append(s, keep);
    return true;
  };
  for (;;) {
    const size_t n = std::fread(buf.data(), 1, buf.size(), in);
    if (n == 0) break;
    w.write(buf.data(), n);
    size_t p = 0;
    if (!carry.empty()) {
      const char* nl = static_cast<const char*>(std::memchr(buf.data(), '\n', n));
      const size_t e = nl ? (size_t)(nl - buf.data()) : n;
      carry.append(buf.data(), e);
      if (!nl) {
        u += n;
        continue;
      }
      take(carry.data(), carry.size(), u - (carry.size() - e));
      carry.clear();
      p = e + 1;
    }
    while (p < n) {
      const char* nl = static_cast<const char*>(std::memchr(buf.data() + p, '\n', n - p));
      if (!nl) {
        carry.assign(buf.data() + p, n - p);
        break;
      }
      const size_t e = (size_t)(nl - buf.data());
      take(buf.data() + p, e - p, u + p);
      p = e + 1;
    }
    u += n;
  }
  std::fclose(in);
  if (!carry.empty()) {  // a last line without '\n' ends at the end of the data
    if (take(carry.data(), carry.size(), u - carry.size())) recs.back().u1 = UINT64_MAX;  // see voff
  }
  w.close();
  uint64_t file_size = 0;
  if (std::FILE* f = std::fopen(output.c_str(), "rb")) {
    std::fseek(f, 0, SEEK_END);
    file_size = (uint64_t)std::ftell(f);
    std::fclose(f);
  }
  auto voff = [&](uint64_t x) -> uint64_t {
    // a last line without '\n': a reader's getline runs on through the EOF
    // block, so tell() is the end of the file
    return x == UINT64_MAX ? file_size << 16 : w.voffset(x);
  };
  TabixBuilder tb(output);
  for (const Rec& r : recs) tb.add(lines.data() + r.at, r.len, voff(r.u0), voff(r.u1));
  tb.write(output + ".tbi");
}

}  // namespace fcsg
