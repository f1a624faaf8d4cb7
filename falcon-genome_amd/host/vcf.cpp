#include "vcf.h"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#include "bam.h"
#include "bgzf.h"
#include "common.h"

namespace fcsg {

std::string VcfRecord::to_line() const {
  std::ostringstream ss;
  ss << chrom << '\t' << pos << '\t' << id << '\t' << ref << '\t';
  if (alts.empty()) ss << '.';
  for (size_t i = 0; i < alts.size(); ++i) ss << (i ? "," : "") << alts[i];
  ss << '\t';
  if (qual < 0) ss << '.';
  else {
    char b[32];
    std::snprintf(b, sizeof b, "%.2f", qual);
    ss << b;
  }
  ss << '\t' << filter << '\t' << info;
  if (!format.empty()) {
    ss << '\t' << format;
    for (const std::string& s : samples) ss << '\t' << s;
  }
  ss << '\n';
  return ss.str();
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
};

VcfWriter::VcfWriter(const std::string& path, const VcfHeader& h) : impl_(new Impl) {
  impl_->out.open(path);
  if (!impl_->out) throw fileNotFound(path + " (cannot write)");
  impl_->out << h.to_text();
}

VcfWriter::~VcfWriter() {
  close();
  delete impl_;
}

void VcfWriter::write(const VcfRecord& r) { impl_->out << r.to_line(); }

void VcfWriter::close() {
  if (impl_->out.is_open()) impl_->out.close();
}

void vcf_concat(const std::vector<std::string>& inputs, const std::string& output) {
  std::ofstream out(output);
  if (!out) throw fileNotFound(output + " (cannot write)");
  for (size_t i = 0; i < inputs.size(); ++i) {
    std::ifstream in(inputs[i]);
    if (!in) throw fileNotFound(inputs[i]);
    std::string line;
    while (std::getline(in, line)) {
      if (!line.empty() && line[0] == '#' && i > 0) continue;
      out << line << '\n';
    }
  }
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

struct RefIndex {
  std::map<uint32_t, std::vector<std::pair<uint64_t, uint64_t>>> bins;
  std::vector<uint64_t> linear;  // 16 kb windows
};

}  // namespace

void tabix_index_vcf(const std::string& vcf_gz) {
  BgzfReader rd(vcf_gz);
  std::vector<std::string> names;
  std::map<std::string, int> name_id;
  std::vector<RefIndex> idx;
  std::string line;
  int last_tid = -1;
  int64_t last_pos = -1;
  for (;;) {
    const uint64_t beg_off = rd.tell();
    if (!rd.getline(line)) break;
    const uint64_t end_off = rd.tell();
    if (line.empty() || line[0] == '#') continue;
    const size_t t1 = line.find('\t'), t2 = line.find('\t', t1 + 1), t3 = line.find('\t', t2 + 1),
                 t4 = line.find('\t', t3 + 1);
    if (t4 == std::string::npos) throw formatError(vcf_gz + ": malformed VCF line");
    const std::string chrom = line.substr(0, t1);
    const int64_t pos = std::stoll(line.substr(t1 + 1, t2 - t1 - 1));
    const int64_t rlen = (int64_t)(t4 - t3 - 1);
    auto it = name_id.find(chrom);
    int tid;
    if (it == name_id.end()) {
      tid = (int)names.size();
      name_id[chrom] = tid;
      names.push_back(chrom);
      idx.emplace_back();
    } else {
      tid = it->second;
      if (tid != last_tid) throw formatError(vcf_gz + ": chromosome blocks not contiguous (unsorted VCF)");
    }
    if (tid == last_tid && pos < last_pos) throw formatError(vcf_gz + ": positions not sorted");
    last_tid = tid;
    last_pos = pos;
    const int64_t beg = pos - 1, end = beg + std::max<int64_t>(rlen, 1);
    RefIndex& ri = idx[tid];
    auto& chunks = ri.bins[reg2bin(beg, end)];
    if (!chunks.empty() && chunks.back().second == beg_off) chunks.back().second = end_off;  // extend the run
    else chunks.emplace_back(beg_off, end_off);
    const int64_t w0 = beg >> 14, w1 = (end - 1) >> 14;
    if ((int64_t)ri.linear.size() <= w1) ri.linear.resize(w1 + 1, 0);
    for (int64_t w = w0; w <= w1; ++w)
      if (ri.linear[w] == 0) ri.linear[w] = beg_off;
  }
  std::string s = "TBI\1";
  put<int32_t>(s, (int32_t)names.size());
  put<int32_t>(s, 2);    // format: VCF
  put<int32_t>(s, 1);    // col_seq
  put<int32_t>(s, 2);    // col_beg
  put<int32_t>(s, 0);    // col_end
  put<int32_t>(s, '#');  // meta char
  put<int32_t>(s, 0);    // skip
  std::string nm;
  for (const std::string& n : names) nm += n + '\0';
  put<int32_t>(s, (int32_t)nm.size());
  s += nm;
  for (RefIndex& ri : idx) {
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
  BgzfWriter w(vcf_gz + ".tbi");
  w.write(s);
  w.close();
}

}  // namespace fcsg
