// Sanitizer driver for the native shard loader (csrc/host/loader.cpp), built by
// tests/test_native_sanitizers_cpu.py with -fsanitize=address,undefined and with
// -fsanitize=thread: many batches in flight on an 8-thread pool (every ticket outstanding at
// once, waited in reverse order), then every gathered record and crop box checked against the
// shard file read independently.  Exit status 0 = all checks passed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../ddp_classification_pytorch_amd/csrc/host/loader.cpp"

namespace {
struct HeaderView {
  char magic[8];
  uint32_t version, channels;
  uint64_t count, index_off, data_off, max_bytes;
};
struct EntryView {
  uint64_t offset;
  uint32_t h, w;
  int64_t label;
};
}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 3;
  std::vector<uint8_t> file;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof(buf), f)) > 0) file.insert(file.end(), buf, buf + k);
  fclose(f);
  HeaderView h;
  memcpy(&h, file.data(), sizeof(h));
  auto entry = [&](int64_t i) {  // memcpy: no alignment assumption about the index in the file
    EntryView e;
    memcpy(&e, file.data() + h.index_off + i * sizeof(EntryView), sizeof(e));
    return e;
  };

  char err[256];
  void* shard = dcpl_open(argv[1], err, sizeof(err));
  if (!shard) {
    fprintf(stderr, "open: %s\n", err);
    return 4;
  }
  if (dcpl_count(shard) != (int64_t)h.count) return 5;
  void* pool = dcpl_pool_create(8);
  const int B = 16, NB = 24;
  std::vector<std::vector<uint8_t>> outs(NB, std::vector<uint8_t>(B * h.max_bytes));
  std::vector<std::vector<int64_t>> metas(NB, std::vector<int64_t>(B * 8)), labels(NB, std::vector<int64_t>(B));
  std::vector<std::vector<int64_t>> order(NB, std::vector<int64_t>(B));
  std::vector<int64_t> tickets(NB);
  for (int b = 0; b < NB; ++b) {
    AugSpec a{b % 3, 40, 32, 0.08f, 1.f, 0.75f, 1.333f, 0.5f};
    for (int i = 0; i < B; ++i) order[b][i] = (b * 7 + i * 3) % (int64_t)h.count;
    tickets[b] = dcpl_submit(pool, shard, order[b].data(), B, outs[b].data(), (int64_t)outs[b].size(), metas[b].data(),
                             labels[b].data(), &a, 1234, (uint64_t)b);
    if (tickets[b] < 0) return 6;
  }
  if (dcpl_wait(pool, 987654321) != -1) return 7;  // unknown ticket
  for (int b = NB - 1; b >= 0; --b)
    if (dcpl_wait(pool, tickets[b]) != 0) return 8;
  int bad = 0;
  for (int b = 0; b < NB; ++b)
    for (int i = 0; i < B; ++i) {
      const EntryView e = entry(order[b][i]);
      const int64_t* m = metas[b].data() + i * 8;
      const size_t nb = (size_t)e.h * e.w * 3;
      if (m[1] != e.h || m[2] != e.w || labels[b][i] != e.label) ++bad;
      if (memcmp(outs[b].data() + m[0], file.data() + h.data_off + e.offset, nb) != 0) ++bad;
      if (m[3] < 0 || m[4] < 0 || m[5] < 1 || m[6] < 1 || m[3] + m[5] > m[1] || m[4] + m[6] > m[2]) ++bad;
    }
  dcpl_pool_destroy(pool);
  dcpl_close(shard);
  if (bad) fprintf(stderr, "%d mismatches\n", bad);
  printf("loader_sanitize ok=%d\n", bad == 0);
  return bad ? 9 : 0;
}
