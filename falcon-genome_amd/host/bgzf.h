// BGZF (blocked gzip) reader and writer on libdeflate (zlib when absent) — the container of BAM,
// bgzipped VCF and tabix indexes (the reference shells
// out to bgzip/tabix/samtools for these, src/worker-htc.cpp:153-176).
//
// Block layout (SAM/BAM spec §4.1): a gzip member with FEXTRA carrying the
// 'BC' subfield (BSIZE = block size - 1), raw-deflate payload of at most 64 KiB,
// CRC32 and ISIZE.  Files end with the fixed 28-byte empty block.  A virtual
// offset is (compressed block start << 16) | offset inside the block.
#pragma once

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <string>
#include <vector>

namespace fcsg {

// Process-wide host worker threads (htslib's thread-pool role): BGZF blocks
// compress here and the one-pass VCF indexer parses its chunks here.  Jobs
// must not wait on other pool jobs.  Workers keep their (thread-local)
// deflate state between blocks.
void host_pool_run(std::function<void()> job);
unsigned host_pool_size();
template <class F>
auto host_pool_async(F f) -> std::future<decltype(f())> {
  auto t = std::make_shared<std::packaged_task<decltype(f())()>>(std::move(f));
  auto fut = t->get_future();
  host_pool_run([t] { (*t)(); });
  return fut;
}

constexpr size_t kBgzfMaxBlock = 0x10000;   // max uncompressed bytes per block
constexpr size_t kBgzfBlockData = 0xff00;   // what the writer packs per block (as htslib)
extern const uint8_t kBgzfEof[28];

// Default deflate level of written BGZF (VCF.gz, BAM).  libdeflate level 5
// against 6 (zlib's and bgzip's default), single thread on this image's
// Xeon: GVCF text 125 vs 85 MB/s at ratio 7.36 vs 7.50; BAM records 142 vs
// 127 MB/s at 2.66 vs 2.67 — the htc tail's bgzip of an 850 MB GVCF is the
// largest single host stage after the shards.  Files differ only in their
// compressed bytes.
constexpr int kBgzfLevel = 5;

class BgzfWriter {
 public:
  explicit BgzfWriter(const std::string& path, int level = kBgzfLevel);
  ~BgzfWriter();
  BgzfWriter(const BgzfWriter&) = delete;
  BgzfWriter& operator=(const BgzfWriter&) = delete;

  void write(const void* data, size_t n);
  void write(const std::string& s) { write(s.data(), s.size()); }
  // Ends the current block so the next write starts a new one (BAM header, index points).
  void flush();
  // Virtual offset of the next byte written.
  uint64_t tell() {
    drain(0);
    return (coff_ << 16) | (uint64_t)buf_.size();
  }
  void close();  // flush + EOF block
  // Compressed start of every block written so far, in order (complete after
  // close()); with no flush() between writes, block k holds the uncompressed
  // bytes [k kBgzfBlockData, (k + 1) kBgzfBlockData).
  const std::vector<uint64_t>& block_offsets() const { return coffs_; }
  // Uncompressed bytes written so far (buffered ones included): a position
  // that voffset() turns into a virtual offset once the writer is closed.
  uint64_t upos() const { return ubytes_; }
  // The virtual offset a BgzfReader's tell() reports at uncompressed position
  // u after reading up to it (a block's end is (that block, its length), not
  // the next block's start).  Valid after close().
  uint64_t voffset(uint64_t u) const;

 private:
  void emit_block(const uint8_t* data, size_t n);
  void drain(size_t keep);  // write finished blocks in order until <= keep are pending
  FILE* f_ = nullptr;
  int level_;
  std::vector<uint8_t> buf_;
  uint64_t coff_ = 0;  // compressed offset of the block being filled (all pending blocks written)
  std::vector<uint64_t> coffs_;
  std::vector<uint64_t> ustarts_;  // uncompressed start of every block, in order
  uint64_t ubytes_ = 0;
  bool closed_ = false;
  bool uniform_ = true;  // every block but the last holds kBgzfBlockData bytes (voffset by division)
  // blocks compress on the host pool and are written in order; tell() first
  // writes every pending block
  std::deque<std::future<std::vector<uint8_t>>> pending_;
  size_t max_pending_ = 0;
};

class BgzfReader {
 public:
  explicit BgzfReader(const std::string& path);
  ~BgzfReader();
  BgzfReader(const BgzfReader&) = delete;
  BgzfReader& operator=(const BgzfReader&) = delete;

  // Reads up to n bytes; returns bytes read (0 at end of data).
  size_t read(void* out, size_t n);
  // Reads exactly n bytes or throws formatError (false when at clean EOF before any byte).
  bool read_exact(void* out, size_t n);
  bool getline(std::string& line);  // text mode ('\n' stripped)
  // The next n bytes in place when they lie inside the current block
  // (consumed; valid until the next read), else nullptr with nothing consumed.
  const uint8_t* view(size_t n) {
    if (pos_ >= block_.size() && !load_block()) return nullptr;
    if (block_.size() - pos_ < n) return nullptr;
    const uint8_t* p = block_.data() + pos_;
    pos_ += n;
    return p;
  }
  uint64_t tell() const;
  void seek(uint64_t voff);
  bool saw_eof_marker() const { return saw_eof_; }
  // Device mode: from the next load on, members are inflated on GPU `device`
  // many at a time (fcs_bgzf_inflate): a load reads a
  // chunk of compressed bytes, inflates every whole member in it in one call
  // and serves their concatenated output as one block, so records spanning
  // members are viewed in place too.  `span` is the caller's estimate of its
  // compressed range from the next seek (a BAI span; 0: unknown): loads cover
  // it in chunks of at most 24 MiB (FCS_BGZF_DEVICE_CHUNK sets every load's
  // size), the next one read and inflated on a helper thread while the caller
  // parses the current one; a chunk goes to the host codec when no warm GPU
  // inflate session is idle (fcs_bgzf_inflate_try).
  void use_device(int device, size_t span);

 private:
  struct Chunk {
    uint64_t start = 0, used = 0;  // file offset, bytes of whole members
    std::vector<uint8_t> comp, out;
    std::vector<int64_t> coff, uoff;  // absolute member offsets, output offsets (n + 1)
    bool empty_member = false;
  };
  bool load_block();  // false at end of file
  bool load_chunk();  // device mode's load_block
  void fetch(uint64_t at, size_t want, Chunk& c);
  size_t first_want() const;
  size_t next_want() const;
  void drop_ahead();
  FILE* f_ = nullptr;
  std::vector<uint8_t> block_, comp_;
  size_t pos_ = 0;
  uint64_t block_coff_ = 0, next_coff_ = 0;
  bool saw_eof_ = false;
  // device mode
  int device_ = -1;
  size_t chunk_ = 0, span_ = 0, want_ = 0;
  uint64_t range_start_ = 0;
  std::vector<int64_t> mcoff_, muoff_;  // the current chunk's members
  Chunk cur_, ahead_;
  std::future<void> ahead_job_;

 public:
  // device mode: chunks inflated on the GPU / on this host (sessions busy)
  int device_chunks() const { return device_chunks_; }
  int host_chunks() const { return host_chunks_; }

 private:
  std::atomic<int> device_chunks_{0}, host_chunks_{0};
};

// Whole-buffer helpers (tests, small files).
std::vector<uint8_t> bgzf_compress(const uint8_t* data, size_t n, int level = kBgzfLevel);
bool is_bgzf_file(const std::string& path);

}  // namespace fcsg
