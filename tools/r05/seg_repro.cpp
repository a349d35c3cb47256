// One P = 1 sort of host-made records through the C ABI of a library given
// by path (dlopen), checked against std::stable_sort on the host: the
// reproducer of stress seed 19 iteration 3258's first half.
//   g++ -O2 -std=c++17 -I include tools/r05/seg_repro.cpp -o tools/r05/seg_repro -ldl
//   tools/r05/seg_repro LIB.so RECORDS.bin HYBRID [REPEAT=1] [OPTION=VALUE ...]
// RECORDS.bin: raw {u64 key, u64 val} records.
#include <dlfcn.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lsb.h"

template <class F>
F sym(void* h, const char* name) {
  void* p = dlsym(h, name);
  if (!p) {
    printf("missing %s\n", name);
    exit(2);
  }
  return reinterpret_cast<F>(p);
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    printf("dlopen: %s\n", dlerror());
    return 2;
  }
  auto create = sym<int (*)(lsb_ctx_t**, int64_t, int, const int*, int)>(h, "lsb_create");
  auto setopt = sym<int (*)(lsb_ctx_t*, int, int64_t)>(h, "lsb_set_option");
  auto cin = sym<int (*)(lsb_ctx_t*, int, int64_t, int64_t, const lsb_elem_t*)>(h, "lsb_copy_in");
  auto cout = sym<int (*)(lsb_ctx_t*, int, int64_t, int64_t, lsb_elem_t*)>(h, "lsb_copy_out");
  auto sort = sym<int (*)(lsb_ctx_t*)>(h, "lsb_sort");
  auto sync = sym<int (*)(lsb_ctx_t*)>(h, "lsb_sync");
  auto destroy = sym<void (*)(lsb_ctx_t*)>(h, "lsb_destroy");
  auto last = sym<int (*)(lsb_ctx_t*, int*, int*, uint64_t*)>(h, "lsb_get_last_sort");
  FILE* f = fopen(argv[2], "rb");
  if (!f) return 2;
  std::vector<lsb_elem_t> in;
  lsb_elem_t e;
  while (fread(&e, sizeof e, 1, f) == 1) in.push_back(e);
  fclose(f);
  const int hybrid = atoi(argv[3]);
  // optional: OPTION=VALUE pairs after REPEAT, set on each context
  std::vector<std::pair<int, long long>> extra;
  for (int i = 5; i < argc; ++i) {
    int o = 0;
    long long v = 0;
    if (sscanf(argv[i], "%d=%lld", &o, &v) == 2) extra.push_back({o, v});
  }
  const int repeat = argc > 4 ? atoi(argv[4]) : 1;
  std::vector<lsb_elem_t> want = in;
  std::stable_sort(want.begin(), want.end(), [](const lsb_elem_t& a, const lsb_elem_t& b) { return a.key < b.key; });
  const int64_t n = (int64_t)in.size();
  int bad_runs = 0;
  for (int k = 0; k < repeat; ++k) {
    lsb_ctx_t* c = nullptr;
    int rc = create(&c, n, 1, nullptr, 8);
    if (rc == 0) rc = setopt(c, LSB_OPT_HYBRID, hybrid);
    for (auto& ov : extra)
      if (rc == 0) rc = setopt(c, ov.first, ov.second);
    if (rc == 0) rc = cin(c, 0, 0, n, in.data());
    if (rc == 0) rc = sort(c);
    if (rc == 0) rc = sync(c);
    std::vector<lsb_elem_t> got(n);
    if (rc == 0) rc = cout(c, 0, 0, n, got.data());
    int lp = -1, ex = -1;
    uint64_t vb = 0;
    if (rc == 0) (void)last(c, &lp, &ex, &vb);
    destroy(c);
    int64_t wrong = 0, first = -1;
    for (int64_t i = 0; i < n; ++i)
      if (got[i].key != want[i].key || got[i].val != want[i].val) {
        if (first < 0) first = i;
        ++wrong;
      }
    printf("run %d: rc %d, n %lld, wrong %lld, first %lld, local passes %d, varying %016llx\n", k, rc, (long long)n,
           (long long)wrong, (long long)first, lp, (unsigned long long)vb);
    bad_runs += wrong != 0 || rc != 0;
  }
  printf("SUMMARY seg_repro %s hybrid %d: %d of %d runs wrong\n", argv[1], hybrid, bad_runs, repeat);
  return bad_runs ? 1 : 0;
}
