// Native batch loader for pre-decoded image shards (host C++, no device code).
//
// Reference behaviour being replaced: the torch DataLoader of BASELINE/main.py:127-131 (4 worker
// processes, each PIL-decoding a JPEG, running RandomResizedCrop(256, scale=(0.8, 1)) /
// Resize(256)+CenterCrop(224) (BASELINE/main.py:58-76) and ToTensor/Normalize on the CPU, then a
// pin-memory thread and `inputs.cuda(non_blocking=True)` (:273-274)).  A handful of host cores
// cannot decode and augment JPEGs at the ~14k img/s one MI355X trains ResNet-50 at, so the work
// is split differently here:
//
//   * images are decoded ONCE, offline, into a shard file of raw uint8 HWC records
//     (`data/shards.py:write_shard`); the loader memory-maps it;
//   * a pool of std::threads gathers the records of one batch (in the order the distributed
//     sampler produced) into a caller-owned pinned buffer and samples each image's augmentation
//     (RandomResizedCrop box with torchvision's 10-attempt algorithm, horizontal flip, or the
//     Resize+CenterCrop box of the eval transform) from a counter-based RNG keyed by
//     (seed, epoch, dataset index), so results do not depend on thread scheduling;
//   * the crop/resize/flip itself runs on the GPU (`dcp::crop_resize_kernel`) after one
//     H2D copy of the raw records, feeding the existing normalise/NHWC input kernel.
//
// C ABI (ctypes, see data/shards.py): dcpl_open / dcpl_close / dcpl_count / dcpl_pool_create /
// dcpl_pool_destroy / dcpl_submit / dcpl_wait.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace {

constexpr char kMagic[8] = {'D', 'C', 'P', 'S', 'H', 'R', 'D', '1'};

#pragma pack(push, 1)
struct Header {        // 48 bytes at offset 0
  char magic[8];
  uint32_t version;    // 1
  uint32_t channels;   // 3
  uint64_t count;
  uint64_t index_off;  // byte offset of `count` IndexEntry records
  uint64_t data_off;   // byte offset of the image records
  uint64_t max_bytes;  // largest record (h*w*c)
};
struct IndexEntry {    // 24 bytes per image
  uint64_t offset;     // relative to data_off
  uint32_t h, w;
  int64_t label;
};
#pragma pack(pop)
static_assert(sizeof(Header) == 48, "header layout");
static_assert(sizeof(IndexEntry) == 24, "index layout");

struct Shard {
  int fd = -1;
  size_t size = 0;
  const uint8_t* base = nullptr;
  const Header* hdr = nullptr;
  const IndexEntry* index = nullptr;
  const uint8_t* data = nullptr;
  ~Shard() {
    if (base) munmap(const_cast<uint8_t*>(base), size);
    if (fd >= 0) close(fd);
  }
};

// Augmentation spec shared with Python (ctypes.Structure in data/shards.py).
struct AugSpec {
  int32_t mode;         // 0 = RandomResizedCrop (+flip), 1 = Resize(resize)+CenterCrop(crop), 2 = whole image
  int32_t resize;       // mode 1: shorter side after resize
  int32_t crop;         // mode 1: centre crop edge (in resized pixels)
  float scale_lo, scale_hi;  // mode 0: area fraction range
  float ratio_lo, ratio_hi;  // mode 0: aspect ratio range
  float flip_p;         // horizontal flip probability (modes 0 and 2)
};

// splitmix64 / counter-based stream: one independent stream per (seed, epoch, dataset index)
struct Rng {
  uint64_t s;
  explicit Rng(uint64_t key) : s(key) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }  // [0, 1)
  int64_t randint(int64_t lo, int64_t hi) {                                 // [lo, hi)
    return lo + static_cast<int64_t>(uniform() * static_cast<double>(hi - lo));
  }
};

inline uint64_t mix_key(uint64_t seed, uint64_t epoch, uint64_t idx) {
  Rng r(seed * 0x100000001B3ull ^ (epoch + 0x51ED27ull) * 0x2545F4914F6CDD1Dull);
  uint64_t a = r.next();
  Rng r2(a ^ (idx * 0xD1B54A32D192ED03ull));
  return r2.next();
}

// torchvision.transforms.RandomResizedCrop.get_params (10 attempts, then the centre fallback).
void rrc_box(Rng& rng, int H, int W, const AugSpec& a, int out[4]) {
  const double area = static_cast<double>(H) * W;
  const double lr0 = std::log(a.ratio_lo), lr1 = std::log(a.ratio_hi);
  for (int t = 0; t < 10; ++t) {
    double target = area * (a.scale_lo + rng.uniform() * (a.scale_hi - a.scale_lo));
    double ar = std::exp(lr0 + rng.uniform() * (lr1 - lr0));
    int w = static_cast<int>(std::lround(std::sqrt(target * ar)));
    int h = static_cast<int>(std::lround(std::sqrt(target / ar)));
    if (w > 0 && h > 0 && w <= W && h <= H) {
      int i = static_cast<int>(rng.randint(0, H - h + 1));
      int j = static_cast<int>(rng.randint(0, W - w + 1));
      out[0] = i, out[1] = j, out[2] = h, out[3] = w;
      return;
    }
  }
  double in_ratio = static_cast<double>(W) / H;
  int w, h;
  if (in_ratio < a.ratio_lo) {
    w = W, h = static_cast<int>(std::lround(w / a.ratio_lo));
  } else if (in_ratio > a.ratio_hi) {
    h = H, w = static_cast<int>(std::lround(h * a.ratio_hi));
  } else {
    w = W, h = H;
  }
  out[0] = (H - h) / 2, out[1] = (W - w) / 2, out[2] = h, out[3] = w;
}

// Resize(shorter side -> resize) + CenterCrop(crop), expressed as a box in source pixels.
void center_box(int H, int W, const AugSpec& a, int out[4]) {
  double s = static_cast<double>(a.resize) / std::min(H, W);  // source -> resized scale
  int ch = std::min(H, static_cast<int>(std::lround(a.crop / s)));
  int cw = std::min(W, static_cast<int>(std::lround(a.crop / s)));
  out[0] = (H - ch) / 2, out[1] = (W - cw) / 2, out[2] = ch, out[3] = cw;
}

class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < std::max(1, n); ++i) threads_.emplace_back([this] { run(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  // Enqueue `n` jobs fn(0..n-1) as one ticket.
  int64_t submit(int n, std::function<int(int)> fn) {
    auto tk = std::make_shared<Ticket>();
    tk->left = n;
    tk->fn = std::move(fn);
    int64_t id;
    {
      std::lock_guard<std::mutex> g(mu_);
      id = next_id_++;
      tickets_[id] = tk;
      for (int i = 0; i < n; ++i) q_.push_back({tk, i});
    }
    cv_.notify_all();
    if (n == 0) {
      std::lock_guard<std::mutex> g(tk->mu);
      tk->done = true;
    }
    return id;
  }
  int wait(int64_t id) {
    std::shared_ptr<Ticket> tk;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto it = tickets_.find(id);
      if (it == tickets_.end()) return -1;
      tk = it->second;
      tickets_.erase(it);
    }
    std::unique_lock<std::mutex> l(tk->mu);
    tk->cv.wait(l, [&] { return tk->done; });
    return tk->err.load();
  }

 private:
  struct Ticket {
    std::mutex mu;
    std::condition_variable cv;
    int left = 0;
    bool done = false;
    std::atomic<int> err{0};
    std::function<int(int)> fn;
  };
  struct Job {
    std::shared_ptr<Ticket> tk;
    int i;
  };
  void run() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        j = q_.front();
        q_.pop_front();
      }
      int rc = j.tk->fn(j.i);
      if (rc != 0) j.tk->err.store(rc);
      std::lock_guard<std::mutex> g(j.tk->mu);
      if (--j.tk->left == 0) {
        j.tk->done = true;
        j.tk->cv.notify_all();
      }
    }
  }
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Job> q_;
  std::map<int64_t, std::shared_ptr<Ticket>> tickets_;
  int64_t next_id_ = 1;
  bool stop_ = false;
};

}  // namespace

extern "C" {

void* dcpl_open(const char* path, char* err, int errlen) {
  auto fail = [&](const std::string& m) -> void* {
    if (err && errlen > 0) snprintf(err, errlen, "%s: %s", path, m.c_str());
    return nullptr;
  };
  auto s = std::make_unique<Shard>();
  s->fd = open(path, O_RDONLY);
  if (s->fd < 0) return fail("cannot open");
  struct stat st;
  if (fstat(s->fd, &st) != 0) return fail("cannot stat");
  s->size = static_cast<size_t>(st.st_size);
  if (s->size < sizeof(Header)) return fail("truncated header");
  void* p = mmap(nullptr, s->size, PROT_READ, MAP_SHARED, s->fd, 0);
  if (p == MAP_FAILED) return fail("mmap failed");
  s->base = static_cast<const uint8_t*>(p);
  s->hdr = reinterpret_cast<const Header*>(s->base);
  const Header& h = *s->hdr;
  if (std::memcmp(h.magic, kMagic, 8) != 0 || h.version != 1 || h.channels != 3) return fail("bad magic/version");
  if (h.index_off + h.count * sizeof(IndexEntry) > s->size || h.data_off > s->size) return fail("truncated index");
  s->index = reinterpret_cast<const IndexEntry*>(s->base + h.index_off);
  s->data = s->base + h.data_off;
  for (uint64_t i = 0; i < h.count; ++i) {
    const IndexEntry& e = s->index[i];
    uint64_t nb = uint64_t(e.h) * e.w * 3;
    if (e.h == 0 || e.w == 0 || nb > h.max_bytes || h.data_off + e.offset + nb > s->size)
      return fail("record " + std::to_string(i) + " out of bounds");
  }
  madvise(p, s->size, MADV_RANDOM);
  return s.release();
}

void dcpl_close(void* shard) { delete static_cast<Shard*>(shard); }

int64_t dcpl_count(void* shard) { return static_cast<int64_t>(static_cast<Shard*>(shard)->hdr->count); }

void* dcpl_pool_create(int nthreads) { return new Pool(nthreads); }

void dcpl_pool_destroy(void* pool) { delete static_cast<Pool*>(pool); }

// Gather the records `indices[0..B)` into `out` (capacity `out_cap` bytes; record b starts at
// b * max_bytes) and write per-image metadata meta[b*8 .. b*8+8) =
// {byte offset in out, H, W, crop y0, crop x0, crop h, crop w, flip}; labels[b] = label.
// Returns a ticket for dcpl_wait (negative on argument errors).
int64_t dcpl_submit(void* pool, void* shard, const int64_t* indices, int B, uint8_t* out, int64_t out_cap,
                    int64_t* meta, int64_t* labels, const AugSpec* aug, uint64_t seed, uint64_t epoch) {
  auto* s = static_cast<Shard*>(shard);
  const uint64_t stride = s->hdr->max_bytes;
  if (B < 0 || static_cast<uint64_t>(B) * stride > static_cast<uint64_t>(out_cap)) return -2;
  for (int b = 0; b < B; ++b)
    if (indices[b] < 0 || static_cast<uint64_t>(indices[b]) >= s->hdr->count) return -3;
  std::vector<int64_t> idx(indices, indices + B);
  AugSpec a = *aug;
  return static_cast<Pool*>(pool)->submit(B, [=](int b) -> int {
    const IndexEntry& e = s->index[idx[b]];
    const int H = static_cast<int>(e.h), W = static_cast<int>(e.w);
    std::memcpy(out + b * stride, s->data + e.offset, size_t(H) * W * 3);
    Rng rng(mix_key(seed, epoch, static_cast<uint64_t>(idx[b])));
    int box[4];
    int flip = 0;
    if (a.mode == 0) {
      rrc_box(rng, H, W, a, box);
      flip = rng.uniform() < a.flip_p;
    } else if (a.mode == 1) {
      center_box(H, W, a, box);
    } else {
      box[0] = 0, box[1] = 0, box[2] = H, box[3] = W;
      flip = rng.uniform() < a.flip_p;
    }
    int64_t* m = meta + b * 8;
    m[0] = static_cast<int64_t>(b * stride);
    m[1] = H, m[2] = W, m[3] = box[0], m[4] = box[1], m[5] = box[2], m[6] = box[3], m[7] = flip;
    labels[b] = e.label;
    return 0;
  });
}

int dcpl_wait(void* pool, int64_t ticket) { return static_cast<Pool*>(pool)->wait(ticket); }

}  // extern "C"
