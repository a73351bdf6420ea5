// Native multi-threaded record loader: the C++ counterpart of task.py's DataLoader(num_workers=8)
// + torchvision transforms (task.py:246-267: RandomCrop(32, padding=4), RandomHorizontalFlip,
// ToTensor, Normalize(mean, std), DistributedSampler shards).
//
// Input: fixed-size binary records, CIFAR-10 binary layout ([label bytes][C planes of H*W
// uint8]); the files are memory-mapped, never read whole.  A pool of worker threads decodes
// whole batches (crop / flip / normalise to float32 NCHW, int64 labels) into a ring of
// `prefetch` batch slots, in order; the consumer copies the next batch into caller memory
// (a pinned host tensor, then one async H2D copy) with the GIL released.
// Augmentation randomness is a pure function of (seed, epoch, sample index), so a resumed or
// re-sharded run sees the same crops/flips for the same sample and epoch.
#include "runtime.hpp"

#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <stdexcept>

namespace mipipe_rt {

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

RecordLoader::RecordLoader(const LoaderConfig& cfg) : cfg_(cfg) {
  if (cfg_.C <= 0 || cfg_.H <= 0 || cfg_.W <= 0 || cfg_.batch <= 0)
    throw std::invalid_argument("bad loader geometry");
  if ((int)cfg_.mean.size() != cfg_.C || (int)cfg_.stdv.size() != cfg_.C)
    throw std::invalid_argument("mean/std must have C entries");
  rec_bytes_ = (size_t)cfg_.label_bytes + (size_t)cfg_.C * cfg_.H * cfg_.W;
  for (auto& f : cfg_.files) {
    int fd = open(f.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) throw std::runtime_error("cannot open " + f);
    struct stat st;
    fstat(fd, &st);
    size_t sz = (size_t)st.st_size;
    if (sz < (size_t)cfg_.header_bytes || (sz - cfg_.header_bytes) % rec_bytes_ != 0) {
      close(fd);
      throw std::runtime_error(f + ": size is not header + k * record_bytes");
    }
    void* p = sz ? mmap(nullptr, sz, PROT_READ, MAP_PRIVATE, fd, 0) : nullptr;
    close(fd);
    if (sz && p == MAP_FAILED) throw std::runtime_error("mmap failed for " + f);
    if (sz) madvise(p, sz, MADV_WILLNEED);
    maps_.push_back({(const uint8_t*)p, sz});
    int64_t n = (int64_t)((sz - cfg_.header_bytes) / rec_bytes_);
    file_start_.push_back(total_);
    total_ += n;
  }
  slot_x_.resize(cfg_.prefetch);
  slot_y_.resize(cfg_.prefetch);
  slot_n_.assign(cfg_.prefetch, 0);
  slot_batch_.assign(cfg_.prefetch, -1);
  const size_t per = (size_t)cfg_.C * cfg_.H * cfg_.W;
  for (int s = 0; s < cfg_.prefetch; ++s) {
    slot_x_[s].resize((size_t)cfg_.batch * per);
    slot_y_[s].resize(cfg_.batch);
  }
  for (int w = 0; w < std::max(1, cfg_.workers); ++w) threads_.emplace_back([this] { worker(); });
}

RecordLoader::~RecordLoader() {
  {
    std::lock_guard<std::mutex> g(mu_);
    shutdown_ = true;
  }
  cv_work_.notify_all();
  cv_slot_.notify_all();
  for (auto& t : threads_) t.join();
  for (auto& m : maps_)
    if (m.first) munmap((void*)m.first, m.second);
}

const uint8_t* RecordLoader::record(int64_t i) const {
  if (i < 0 || i >= total_) throw std::out_of_range("record index");
  size_t f = std::upper_bound(file_start_.begin(), file_start_.end(), i) - file_start_.begin() - 1;
  return maps_[f].first + cfg_.header_bytes + (size_t)(i - file_start_[f]) * rec_bytes_;
}

void RecordLoader::start_epoch(const std::vector<int64_t>& indices, int64_t epoch) {
  for (int64_t i : indices)
    if (i < 0 || i >= total_) throw std::out_of_range("sampler index out of range");
  std::unique_lock<std::mutex> g(mu_);
  ++gen_;  // workers drop batches of the previous generation
  cv_slot_.wait(g, [this] { return busy_ == 0; });
  indices_ = indices;
  epoch_ = epoch;
  const int64_t n = (int64_t)indices_.size();
  nbatches_ = cfg_.drop_last ? n / cfg_.batch : (n + cfg_.batch - 1) / cfg_.batch;
  next_produce_ = 0;
  next_consume_ = 0;
  std::fill(slot_batch_.begin(), slot_batch_.end(), -1);
  g.unlock();
  cv_work_.notify_all();
}

void RecordLoader::fill(int slot, int64_t b, const std::vector<int64_t>& idx, int64_t epoch) {
  const int C = cfg_.C, H = cfg_.H, W = cfg_.W, P = cfg_.pad;
  const int64_t i0 = b * cfg_.batch;
  const int n = (int)std::min<int64_t>(cfg_.batch, (int64_t)idx.size() - i0);
  float* xo = slot_x_[slot].data();
  int64_t* yo = slot_y_[slot].data();
  const size_t plane = (size_t)H * W;
  for (int s = 0; s < n; ++s) {
    const int64_t gi = idx[i0 + s];
    const uint8_t* r = record(gi);
    int64_t label = 0;
    for (int k = 0; k < cfg_.label_bytes; ++k) label |= (int64_t)r[k] << (8 * k);
    yo[s] = label;
    const uint8_t* img = r + cfg_.label_bytes;
    int dy = 0, dx = 0;
    bool flip = false;
    if (cfg_.train) {
      uint64_t h = splitmix64(cfg_.seed ^ splitmix64((uint64_t)epoch * 0x100000001b3ull ^ (uint64_t)gi));
      if (P > 0) {
        dy = (int)(h % (uint64_t)(2 * P + 1)) - P;
        dx = (int)((h >> 16) % (uint64_t)(2 * P + 1)) - P;
      }
      flip = cfg_.flip && ((h >> 40) & 1);
    }
    float* xs = xo + (size_t)s * C * plane;
    for (int c = 0; c < C; ++c) {
      const float sc = 1.f / (255.f * cfg_.stdv[c]);
      const float off = -cfg_.mean[c] / cfg_.stdv[c];
      const uint8_t* ip = img + (size_t)c * plane;
      float* op = xs + (size_t)c * plane;
      for (int y = 0; y < H; ++y) {
        const int sy = y + dy;
        for (int x = 0; x < W; ++x) {
          const int xx = flip ? W - 1 - x : x;
          const int sx = xx + dx;
          // zero padding (RandomCrop(padding=P) pads the uint8 image with 0)
          const float v = (sy >= 0 && sy < H && sx >= 0 && sx < W) ? (float)ip[sy * W + sx] : 0.f;
          op[y * W + x] = v * sc + off;
        }
      }
    }
  }
  slot_n_[slot] = n;
}

void RecordLoader::worker() {
  std::unique_lock<std::mutex> g(mu_);
  while (true) {
    cv_work_.wait(g, [this] {
      return shutdown_ || (next_produce_ < nbatches_ && next_produce_ - next_consume_ < cfg_.prefetch);
    });
    if (shutdown_) return;
    const int64_t b = next_produce_++;
    const int slot = (int)(b % cfg_.prefetch);
    const uint64_t gen = gen_;
    const std::vector<int64_t>* idx = &indices_;
    const int64_t epoch = epoch_;
    ++busy_;
    g.unlock();
    fill(slot, b, *idx, epoch);
    g.lock();
    --busy_;
    if (gen == gen_) slot_batch_[slot] = b;
    cv_slot_.notify_all();
  }
}

int RecordLoader::next(float* x, int64_t* y) {
  std::unique_lock<std::mutex> g(mu_);
  if (next_consume_ >= nbatches_) return 0;
  const int64_t b = next_consume_;
  const int slot = (int)(b % cfg_.prefetch);
  cv_slot_.wait(g, [&] { return slot_batch_[slot] == b || shutdown_; });
  if (shutdown_) return 0;
  const int n = slot_n_[slot];
  g.unlock();
  const size_t per = (size_t)cfg_.C * cfg_.H * cfg_.W;
  memcpy(x, slot_x_[slot].data(), (size_t)n * per * sizeof(float));
  memcpy(y, slot_y_[slot].data(), (size_t)n * sizeof(int64_t));
  g.lock();
  slot_batch_[slot] = -1;
  ++next_consume_;
  g.unlock();
  cv_work_.notify_all();
  return n;
}

int64_t RecordLoader::batches_per_epoch() const { return nbatches_; }

}  // namespace mipipe_rt
