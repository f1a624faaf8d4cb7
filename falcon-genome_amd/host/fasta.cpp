#include "fasta.h"

#include <array>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>

#include "common.h"

namespace fcsg {

int Reference::index(const std::string& name) const {
  for (size_t i = 0; i < contigs.size(); ++i)
    if (contigs[i].name == name) return (int)i;
  return -1;
}

int64_t Reference::total_length() const {
  int64_t n = 0;
  for (const Contig& c : contigs) n += (int64_t)c.seq.size();
  return n;
}

Reference load_fasta(const std::string& path) {
  // the whole file in one read, then one pass over its lines: bases through a
  // 256-entry table (upper case ACGT kept, anything else N), a line's bases
  // appended in one copy
  std::FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw fileNotFound(path);
  std::string buf;
  {
    char chunk[1 << 16];
    size_t got;
    if (std::fseek(f, 0, SEEK_END) == 0) {
      const long n = std::ftell(f);
      if (n > 0) buf.reserve((size_t)n);
      std::fseek(f, 0, SEEK_SET);
    }
    while ((got = std::fread(chunk, 1, sizeof chunk, f)) > 0) buf.append(chunk, got);
    std::fclose(f);
  }
  static const auto kBase = [] {
    std::array<char, 256> t{};
    for (int c = 0; c < 256; ++c) {
      const int u = std::toupper(c);
      t[c] = (u == 'A' || u == 'C' || u == 'G' || u == 'T') ? (char)u : 'N';
    }
    return t;
  }();
  Reference ref;
  std::string* s = nullptr;
  const char* p = buf.data();
  const char* const e = p + buf.size();
  while (p < e) {
    const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
    const char* le = nl ? nl : e;
    const char* q = le;
    if (q > p && q[-1] == '\r') --q;
    if (q > p) {
      if (*p == '>') {
        std::string name(p + 1, q);
        const size_t ws = name.find_first_of(" \t");
        if (ws != std::string::npos) name.resize(ws);
        ref.contigs.push_back({name, ""});
        s = &ref.contigs.back().seq;
      } else {
        if (!s) throw formatError(path + ": sequence before the first '>' header");
        const size_t at = s->size();
        s->resize(at + (size_t)(q - p));
        char* o = &(*s)[at];
        for (const char* c = p; c < q; ++c) *o++ = kBase[(unsigned char)*c];
      }
    }
    p = nl ? nl + 1 : e;
  }
  return ref;
}

void write_fasta(const std::string& path, const Reference& ref, int lw) {
  std::ofstream out(path);
  if (!out) throw fileNotFound(path + " (cannot write)");
  for (const Contig& c : ref.contigs) {
    out << '>' << c.name << '\n';
    for (size_t k = 0; k < c.seq.size(); k += lw) out << c.seq.substr(k, lw) << '\n';
  }
}

void write_fai(const std::string& fasta_path, const Reference& ref, int lw) {
  std::ofstream out(fasta_path + ".fai");
  int64_t off = 0;
  for (const Contig& c : ref.contigs) {
    off += 1 + (int64_t)c.name.size() + 1;  // ">name\n"
    out << c.name << '\t' << c.seq.size() << '\t' << off << '\t' << lw << '\t' << lw + 1 << '\n';
    const int64_t L = (int64_t)c.seq.size();
    off += L + (L + lw - 1) / lw;  // bases + one newline per line
  }
}

void write_dict(const std::string& dict_path, const Reference& ref) {
  std::ofstream out(dict_path);
  out << "@HD\tVN:1.6\tSO:unsorted\n";
  for (const Contig& c : ref.contigs) out << "@SQ\tSN:" << c.name << "\tLN:" << c.seq.size() << '\n';
}

std::string dict_path_for(const std::string& ref_path) {
  const size_t slash = ref_path.find_last_of('/');
  const size_t dot = ref_path.find_last_of('.');
  if (dot == std::string::npos || (slash != std::string::npos && dot < slash)) return ref_path + ".dict";
  return ref_path.substr(0, dot) + ".dict";
}

std::vector<std::pair<std::string, int64_t>> read_dict(const std::string& dict_path) {
  std::ifstream in(dict_path);
  if (!in) throw fileNotFound(dict_path);
  std::vector<std::pair<std::string, int64_t>> out;
  std::string line;
  while (std::getline(in, line)) {
    if (line.compare(0, 3, "@SQ") != 0) continue;
    std::istringstream ss(line);
    std::string tok, name;
    int64_t len = -1;
    while (ss >> tok) {
      if (tok.compare(0, 3, "SN:") == 0) name = tok.substr(3);
      else if (tok.compare(0, 3, "LN:") == 0) len = std::stoll(tok.substr(3));
    }
    if (name.empty() || len < 0) throw formatError(dict_path + ": malformed @SQ line");
    out.emplace_back(name, len);
  }
  return out;
}

}  // namespace fcsg
