#include "bgzf.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "common.h"
#include "fcship.h"

namespace fcsg {

const uint8_t kBgzfEof[28] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0, 0x42, 0x43,
                              0x02, 0,    0x1b, 0,    3, 0, 0, 0, 0, 0, 0,    0, 0, 0};

namespace {

void put16(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
}
void put32(uint8_t* p, uint32_t v) {
  for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
uint32_t get16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
uint32_t get32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// The raw-deflate codec.  libdeflate (the image's libdeflate.so.0, the codec
// htslib prefers when built with it) inflates and deflates whole 64 KiB
// blocks in one call, about twice zlib's speed; it is opened at run time and
// zlib stays the codec when it is absent or FCS_BGZF_ZLIB=1.  Either codec's
// output is a valid raw-deflate stream, so files differ only in the
// compressed bytes, never in content.
struct Libdeflate {
  void* (*alloc_decompressor)() = nullptr;
  int (*deflate_decompress)(void*, const void*, size_t, void*, size_t, size_t*) = nullptr;
  void (*free_decompressor)(void*) = nullptr;
  void* (*alloc_compressor)(int) = nullptr;
  size_t (*deflate_compress)(void*, const void*, size_t, void*, size_t) = nullptr;
  void (*free_compressor)(void*) = nullptr;
  uint32_t (*crc32)(uint32_t, const void*, size_t) = nullptr;
  bool ok = false;
};

const Libdeflate& libdeflate() {
  static const Libdeflate L = [] {
    Libdeflate l;
    const char* force = std::getenv("FCS_BGZF_ZLIB");
    if (force && *force && *force != '0') return l;
    void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
    if (!h) return l;
    auto sym = [&](auto& f, const char* name) { f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name)); };
    sym(l.alloc_decompressor, "libdeflate_alloc_decompressor");
    sym(l.deflate_decompress, "libdeflate_deflate_decompress");
    sym(l.free_decompressor, "libdeflate_free_decompressor");
    sym(l.alloc_compressor, "libdeflate_alloc_compressor");
    sym(l.deflate_compress, "libdeflate_deflate_compress");
    sym(l.free_compressor, "libdeflate_free_compressor");
    sym(l.crc32, "libdeflate_crc32");
    l.ok = l.alloc_decompressor && l.deflate_decompress && l.free_decompressor && l.alloc_compressor &&
           l.deflate_compress && l.free_compressor && l.crc32;
    return l;
  }();
  return L;
}

uint32_t block_crc(const uint8_t* p, size_t n) {
  const Libdeflate& L = libdeflate();
  return L.ok ? L.crc32(0, p, n) : (uint32_t)crc32(crc32(0L, Z_NULL, 0), p, (uInt)n);
}

// Raw inflate of a whole block into out[0, isize); false when corrupt.
bool inflate_block(const uint8_t* in, size_t n, uint8_t* out, size_t isize) {
  const Libdeflate& L = libdeflate();
  if (L.ok) {
    struct Free {
      void operator()(void* d) const { libdeflate().free_decompressor(d); }
    };
    thread_local std::unique_ptr<void, Free> dec(L.alloc_decompressor());
    if (!dec) throw internalError("[E::bgzf] libdeflate_alloc_decompressor failed");
    size_t got = 0;
    return L.deflate_decompress(dec.get(), in, n, out, isize, &got) == 0 && got == isize;
  }
  z_stream zs{};
  if (inflateInit2(&zs, -15) != Z_OK) throw internalError("[E::bgzf] inflateInit2 failed");
  zs.next_in = const_cast<uint8_t*>(in);
  zs.avail_in = (uInt)n;
  zs.next_out = out;
  zs.avail_out = (uInt)isize;
  const int rc = inflate(&zs, Z_FINISH);
  inflateEnd(&zs);
  return rc == Z_STREAM_END && zs.total_out == isize;
}

// Raw deflate of data[0, n) into out[0, cap) at `level`; 0 when it does not fit.
size_t deflate_block(const uint8_t* data, size_t n, uint8_t* out, size_t cap, int level) {
  const Libdeflate& L = libdeflate();
  if (L.ok && level > 0) {
    struct Free {
      void operator()(void* c) const { libdeflate().free_compressor(c); }
    };
    thread_local int tl_level = -1;
    thread_local std::unique_ptr<void, Free> comp;
    if (tl_level != level) {
      comp.reset(L.alloc_compressor(std::min(level, 12)));
      if (!comp) throw internalError("[E::bgzf] libdeflate_alloc_compressor failed");
      tl_level = level;
    }
    return L.deflate_compress(comp.get(), data, n, out, cap);
  }
  z_stream zs{};
  if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    throw internalError("[E::bgzf] deflateInit2 failed");
  zs.next_in = const_cast<uint8_t*>(data);
  zs.avail_in = (uInt)n;
  zs.next_out = out;
  zs.avail_out = (uInt)cap;
  const int rc = deflate(&zs, Z_FINISH);
  const size_t clen = zs.total_out;
  deflateEnd(&zs);
  return rc == Z_STREAM_END ? clen : 0;
}

// One BGZF member for n <= kBgzfMaxBlock input bytes.
std::vector<uint8_t> make_block(const uint8_t* data, size_t n, int level) {
  std::vector<uint8_t> out(kBgzfMaxBlock + 64);
  for (int attempt = 0; attempt < 2; ++attempt) {
    const size_t clen = deflate_block(data, n, out.data() + 18, kBgzfMaxBlock - 18 - 8, attempt ? 0 : level);
    if (clen == 0) {
      if (attempt == 0) continue;  // incompressible: store (level 0) instead
      throw internalError("[E::bgzf] block does not fit in 64 KiB");
    }
    const size_t bsize = 18 + clen + 8;
    static const uint8_t hdr[16] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0, 0x42, 0x43, 0x02, 0};
    std::memcpy(out.data(), hdr, 16);
    put16(out.data() + 16, (uint32_t)(bsize - 1));
    put32(out.data() + 18 + clen, block_crc(data, n));
    put32(out.data() + 18 + clen + 4, (uint32_t)n);
    out.resize(bsize);
    return out;
  }
  return {};
}

}  // namespace

// ------------------------------------------------------------------ pool
namespace {

class HostPool {
 public:
  HostPool() {
    n_ = host_cpus();
    for (unsigned k = 0; k < n_; ++k) threads_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : threads_) t.join();
  }
  void run(std::function<void()> job) {
    {
      std::lock_guard<std::mutex> g(mu_);
      jobs_.push_back(std::move(job));
    }
    cv_.notify_one();
  }
  unsigned size() const { return n_; }

 private:
  void loop() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !jobs_.empty(); });
        if (jobs_.empty()) return;  // stop_ with nothing left
        job = std::move(jobs_.front());
        jobs_.pop_front();
      }
      job();  // packaged tasks keep their exceptions for the waiter
    }
  }
  unsigned n_ = 1;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> jobs_;
  std::vector<std::thread> threads_;
  bool stop_ = false;
};

HostPool& host_pool() {
  static HostPool p;
  return p;
}

}  // namespace

void host_pool_run(std::function<void()> job) { host_pool().run(std::move(job)); }
unsigned host_pool_size() { return host_pool().size(); }

// ------------------------------------------------------------------ writer
BgzfWriter::BgzfWriter(const std::string& path, int level) : level_(level) {
  f_ = std::fopen(path.c_str(), "wb");
  if (!f_) throw fileNotFound(path + " (cannot open for writing)");
  buf_.reserve(kBgzfMaxBlock);
  max_pending_ = 4 * (size_t)host_pool_size();
}

BgzfWriter::~BgzfWriter() {
  try {
    close();
  } catch (...) {
  }
}

void BgzfWriter::emit_block(const uint8_t* data, size_t n) {
  ustarts_.push_back(ubytes_ - n);
  std::vector<uint8_t> in(data, data + n);
  const int level = level_;
  pending_.push_back(host_pool_async([in = std::move(in), level] { return make_block(in.data(), in.size(), level); }));
  drain(max_pending_);
}

void BgzfWriter::drain(size_t keep) {
  while (pending_.size() > keep) {
    const std::vector<uint8_t> blk = pending_.front().get();
    pending_.pop_front();
    if (std::fwrite(blk.data(), 1, blk.size(), f_) != blk.size()) throw internalError("[E::bgzf] write failed");
    coffs_.push_back(coff_);
    coff_ += blk.size();
  }
}

void BgzfWriter::write(const void* data, size_t n) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  while (n > 0) {
    const size_t take = std::min(n, kBgzfBlockData - buf_.size());
    buf_.insert(buf_.end(), p, p + take);
    ubytes_ += take;
    p += take;
    n -= take;
    if (buf_.size() >= kBgzfBlockData) flush();
  }
}

void BgzfWriter::flush() {
  if (buf_.empty()) return;
  if (buf_.size() != kBgzfBlockData) uniform_ = false;  // a short block before more data
  emit_block(buf_.data(), buf_.size());
  buf_.clear();
}

void BgzfWriter::close() {
  if (closed_ || !f_) return;
  if (!buf_.empty()) {  // the last block may be short without breaking uniform_
    emit_block(buf_.data(), buf_.size());
    buf_.clear();
  }
  drain(0);
  std::fwrite(kBgzfEof, 1, sizeof kBgzfEof, f_);
  std::fclose(f_);
  f_ = nullptr;
  closed_ = true;
}

uint64_t BgzfWriter::voffset(uint64_t u) const {
  if (!closed_ || coffs_.size() != ustarts_.size()) throw internalError("[E::bgzf] voffset before close");
  if (ustarts_.empty()) return 0;
  size_t k;
  if (uniform_)
    k = std::min<size_t>((size_t)(u / kBgzfBlockData), ustarts_.size() - 1);  // block k starts at k kBgzfBlockData
  else
    k = (size_t)(std::upper_bound(ustarts_.begin(), ustarts_.end(), u) - ustarts_.begin()) - 1;
  if (k > 0 && u == ustarts_[k]) --k;  // a block boundary reached by reading: the end of the earlier block
  return (coffs_[k] << 16) | (u - ustarts_[k]);
}

// ------------------------------------------------------------------ reader
BgzfReader::BgzfReader(const std::string& path) {
  f_ = std::fopen(path.c_str(), "rb");
  if (!f_) throw fileNotFound(path);
  std::setvbuf(f_, nullptr, _IOFBF, 1 << 20);  // about 30 blocks per read(2)
}

namespace {
// Device mode's chunk buffers outlive a reader on its thread: a window's
// chunk is tens of MiB, and fresh buffers for every window cost a page fault
// per 4 KiB of it.
struct ChunkCache {
  std::vector<uint8_t> comp, out, block;
};
ChunkCache& chunk_cache() {
  static thread_local ChunkCache c;
  return c;
}
}  // namespace

BgzfReader::~BgzfReader() {
  drop_ahead();  // the helper thread reads f_
  if (f_) std::fclose(f_);
  if (device_ >= 0) {
    ChunkCache& c = chunk_cache();
    c.comp.swap(cur_.comp);
    c.out.swap(cur_.out);
    c.block.swap(block_);
  }
}

bool BgzfReader::load_block() {
  if (device_ >= 0) return load_chunk();
  for (;;) {
    block_coff_ = next_coff_;
    // sequential blocks need no seek (a seek drops the stdio buffer)
    if (std::ftell(f_) != (long)block_coff_ && std::fseek(f_, (long)block_coff_, SEEK_SET) != 0) return false;
    uint8_t h[18];
    const size_t got = std::fread(h, 1, 18, f_);
    if (got == 0) return false;
    if (got < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8 || !(h[3] & 4))
      throw formatError("not a BGZF block at offset " + std::to_string(block_coff_));
    const uint32_t xlen = get16(h + 10);
    // find the BC subfield (it is the only one we write; others are skipped)
    std::vector<uint8_t> extra(xlen);
    std::memcpy(extra.data(), h + 12, std::min<uint32_t>(xlen, 6));
    if (xlen > 6 && std::fread(extra.data() + 6, 1, xlen - 6, f_) != xlen - 6) throw formatError("truncated BGZF header");
    uint32_t bsize = 0;
    for (uint32_t k = 0; k + 4 <= xlen;) {
      const uint32_t slen = get16(&extra[k + 2]);
      if (extra[k] == 66 && extra[k + 1] == 67 && slen == 2) bsize = get16(&extra[k + 4]) + 1;
      k += 4 + slen;
    }
    if (bsize == 0) throw formatError("gzip member without BGZF BC field");
    const size_t hdr = 12 + xlen;
    if (bsize < hdr + 8) throw formatError("corrupt BGZF block header");
    // the header is read; the rest of the member follows it in the file
    std::vector<uint8_t>& comp = comp_;
    comp.resize(bsize);
    std::memcpy(comp.data(), h, 12);
    std::memcpy(comp.data() + 12, extra.data(), xlen);
    if (std::fread(comp.data() + hdr, 1, bsize - hdr, f_) != bsize - hdr) throw formatError("truncated BGZF block");
    const uint32_t isize = get32(&comp[bsize - 4]);
    const uint32_t crc = get32(&comp[bsize - 8]);
    if (isize > kBgzfMaxBlock || bsize < hdr + 8) throw formatError("corrupt BGZF block header");
    block_.resize(isize);
    if (isize > 0) {
      if (!inflate_block(comp.data() + hdr, bsize - hdr - 8, block_.data(), isize))
        throw formatError("corrupt BGZF block payload");
      if (block_crc(block_.data(), isize) != crc) throw formatError("BGZF CRC mismatch");
    }
    next_coff_ = block_coff_ + bsize;
    pos_ = 0;
    if (isize == 0) {
      saw_eof_ = true;  // empty block (EOF marker, or an empty block mid-file): keep going
      continue;
    }
    return true;
  }
}

size_t BgzfReader::read(void* out, size_t n) {
  uint8_t* o = static_cast<uint8_t*>(out);
  size_t done = 0;
  while (done < n) {
    if (pos_ >= block_.size() && !load_block()) break;
    const size_t take = std::min(n - done, block_.size() - pos_);
    std::memcpy(o + done, block_.data() + pos_, take);
    pos_ += take;
    done += take;
  }
  return done;
}

bool BgzfReader::read_exact(void* out, size_t n) {
  const size_t got = read(out, n);
  if (got == 0 && n > 0) return false;
  if (got != n) throw formatError("truncated BGZF data");
  return true;
}

bool BgzfReader::getline(std::string& line) {
  line.clear();
  bool any = false;
  for (;;) {
    if (pos_ >= block_.size() && !load_block()) return any;
    any = true;
    const uint8_t* s = block_.data() + pos_;
    const uint8_t* e = block_.data() + block_.size();
    const uint8_t* nl = static_cast<const uint8_t*>(std::memchr(s, '\n', e - s));
    if (nl) {
      line.append(reinterpret_cast<const char*>(s), nl - s);
      pos_ += (nl - s) + 1;
      return true;
    }
    line.append(reinterpret_cast<const char*>(s), e - s);
    pos_ = block_.size();
  }
}

uint64_t BgzfReader::tell() const {
  if (mcoff_.size() < 2) return (block_coff_ << 16) | (uint64_t)pos_;
  // the chunk's member holding pos_; a member boundary reached by reading is
  // the end of the earlier member, as for single blocks
  size_t k = (size_t)(std::upper_bound(muoff_.begin(), muoff_.end() - 1, (int64_t)pos_) - muoff_.begin()) - 1;
  if (k > 0 && (int64_t)pos_ == muoff_[k]) --k;
  return ((uint64_t)mcoff_[k] << 16) | (uint64_t)(pos_ - (size_t)muoff_[k]);
}

void BgzfReader::use_device(int device, size_t span) {
  if (device_ < 0) {  // reuse this thread's buffers of an earlier reader
    ChunkCache& c = chunk_cache();
    cur_.comp.swap(c.comp);
    cur_.out.swap(c.out);
    if (block_.empty()) {  // (a block still being read stays)
      block_.swap(c.block);
      block_.clear();
      pos_ = 0;
    }
  }
  device_ = device;
  chunk_ = 24u << 20;
  if (const char* e = std::getenv("FCS_BGZF_DEVICE_CHUNK"); e && std::atoll(e) > 0) chunk_ = (size_t)std::atoll(e);
  chunk_ = std::max<size_t>(chunk_, 1 << 17);  // two whole members at least
  span_ = span;
  range_start_ = next_coff_;
  want_ = first_want();
}

// The first load after a seek covers the caller's whole estimated range in
// one call (the kernel's rate comes from many members in flight: a shard's
// range is a few hundred members, a chunk of it a few dozen), at most 256 MiB.
size_t BgzfReader::first_want() const { return next_want(); }

// Inside the caller's range: the rest of it, at most chunk_ (24 MiB: the
// inflate sessions' staging holds such a chunk with its output); past it
// 1 MiB loads finish the reads that start inside the range.
size_t BgzfReader::next_want() const {
  if (std::getenv("FCS_BGZF_DEVICE_CHUNK")) return chunk_;
  const uint64_t done = next_coff_ - range_start_;
  if (!span_) return chunk_;
  if (done < span_) return std::min<size_t>(std::max<size_t>(span_ - (size_t)done, 1 << 17), chunk_);
  return 1 << 20;
}

// Reads `want` bytes at `at` and inflates their whole members into c.
void BgzfReader::fetch(uint64_t at, size_t want, Chunk& c) {
  c.start = at;
  c.used = 0;
  c.empty_member = false;  // (c.out keeps its size: a resize below fills only what it adds)
  if (std::ftell(f_) != (long)at && std::fseek(f_, (long)at, SEEK_SET) != 0) return;
  c.comp.resize(want);
  const size_t got = std::fread(c.comp.data(), 1, want, f_);
  if (got == 0) return;
  const size_t cap = got / 20 + 2;
  c.coff.resize(cap + 1);
  c.uoff.resize(cap + 1);
  int32_t n = 0;
  int64_t used = 0;
  if (fcs_bgzf_index(c.comp.data(), (int64_t)got, c.coff.data(), c.uoff.data(), (int32_t)cap, &n, &used) != FCS_OK)
    throw formatError(std::string("BGZF at offset ") + std::to_string(at) + ": " + fcs_last_error());
  if (n == 0) throw formatError("truncated BGZF block at offset " + std::to_string(at));
  c.coff.resize((size_t)n + 1);
  c.uoff.resize((size_t)n + 1);
  c.out.resize((size_t)c.uoff[(size_t)n]);
  int64_t used2 = 0, out = 0;
  // the GPU when one of its inflate sessions is idle and warm, else this
  // thread's libdeflate: a reader never queues behind other shards' calls
  const int rc = fcs_bgzf_inflate_try(c.comp.data(), used, c.out.data(), (int64_t)c.out.size(), &used2, &out, device_);
  if (rc == FCS_BGZF_BUSY) {
    ++host_chunks_;
    for (int32_t k = 0; k < n; ++k) {
      const uint8_t* m = c.comp.data() + c.coff[(size_t)k];
      const size_t len = (size_t)(c.coff[(size_t)k + 1] - c.coff[(size_t)k]), hdr = 12 + get16(m + 10);
      const size_t isize = (size_t)(c.uoff[(size_t)k + 1] - c.uoff[(size_t)k]);
      uint8_t* o = c.out.data() + c.uoff[(size_t)k];
      if (isize && (!inflate_block(m + hdr, len - hdr - 8, o, isize) || block_crc(o, isize) != get32(m + len - 8)))
        throw formatError("corrupt BGZF block at offset " + std::to_string(at + (uint64_t)c.coff[(size_t)k]));
    }
  } else if (rc != FCS_OK) {
    throw formatError(std::string("BGZF at offset ") + std::to_string(at) + ": " + fcs_last_error());
  } else {
    ++device_chunks_;
  }
  for (int32_t k = 0; k <= n; ++k) c.coff[(size_t)k] += (int64_t)at;
  for (int32_t k = 0; k < n; ++k)
    if (c.uoff[(size_t)k + 1] == c.uoff[(size_t)k]) c.empty_member = true;  // the EOF marker
  c.used = (uint64_t)used;
}

void BgzfReader::drop_ahead() {
  if (!ahead_job_.valid()) return;
  try {
    ahead_job_.get();
  } catch (...) {  // a prefetch past the caller's range may fail; it is not used
  }
}

bool BgzfReader::load_chunk() {
  for (;;) {
    if (ahead_job_.valid()) {
      ahead_job_.get();  // a failure of the chunk the caller needs is reported here
      std::swap(cur_, ahead_);
    } else {
      fetch(next_coff_, want_, cur_);
    }
    want_ = 0;  // (set from the new position below)
    if (cur_.used == 0) return false;
    block_.swap(cur_.out);
    mcoff_.swap(cur_.coff);
    muoff_.swap(cur_.uoff);
    block_coff_ = cur_.start;
    next_coff_ = cur_.start + cur_.used;
    want_ = next_want();
    saw_eof_ = saw_eof_ || cur_.empty_member;
    pos_ = 0;
    // the next chunk on a helper thread while the caller parses this one,
    // inside the caller's estimated range only
    if (!span_ || next_coff_ - range_start_ < span_)
      ahead_job_ = std::async(std::launch::async, [this, at = next_coff_, w = want_] { fetch(at, w, ahead_); });
    if (!block_.empty()) return true;
  }
}

void BgzfReader::seek(uint64_t voff) {
  drop_ahead();
  next_coff_ = voff >> 16;
  block_.clear();
  mcoff_.clear();
  muoff_.clear();
  if (device_ >= 0) {
    range_start_ = next_coff_;
    want_ = first_want();
  }
  pos_ = 0;
  if (!load_block()) throw formatError("seek past end of BGZF file");
  pos_ = (size_t)(voff & 0xffff);
}

std::vector<uint8_t> bgzf_compress(const uint8_t* data, size_t n, int level) {
  std::vector<uint8_t> out;
  for (size_t k = 0; k < n; k += kBgzfBlockData) {
    const std::vector<uint8_t> b = make_block(data + k, std::min(kBgzfBlockData, n - k), level);
    out.insert(out.end(), b.begin(), b.end());
  }
  out.insert(out.end(), kBgzfEof, kBgzfEof + sizeof kBgzfEof);
  return out;
}

bool is_bgzf_file(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  uint8_t h[16];
  const bool ok = std::fread(h, 1, 16, f) == 16 && h[0] == 0x1f && h[1] == 0x8b && (h[3] & 4) && h[12] == 66 &&
                  h[13] == 67;
  std::fclose(f);
  return ok;
}

}  // namespace fcsg
