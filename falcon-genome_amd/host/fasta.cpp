#include "fasta.h"

#include <cctype>
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
  std::ifstream in(path);
  if (!in) throw fileNotFound(path);
  Reference ref;
  std::string line;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    if (line[0] == '>') {
      std::string name = line.substr(1);
      const size_t ws = name.find_first_of(" \t");
      if (ws != std::string::npos) name.resize(ws);
      ref.contigs.push_back({name, ""});
      continue;
    }
    if (ref.contigs.empty()) throw formatError(path + ": sequence before the first '>' header");
    std::string& s = ref.contigs.back().seq;
    for (char c : line) {
      const char u = (char)std::toupper((unsigned char)c);
      s += (u == 'A' || u == 'C' || u == 'G' || u == 'T') ? u : 'N';
    }
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
