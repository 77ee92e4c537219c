// =============================================================================
//  kat.cpp — TEST INFRASTRUCTURE ONLY.
//
//  Known-answer tests that pin the CPU oracle (lkf_oracle.h) to the reference's
//  own unit tests.  The Go reference cannot be built here (no Go toolchain,
//  SURVEY.md §8(c)), so each reference test's inputs and expected values are
//  transcribed as data below, citing the test file:line they come from
//  (relative to /root/reference/pkg/sfu).  The checks run against the oracle's
//  restatement; a mismatch means the oracle (and therefore every GPU parity
//  claim built on it) diverges from the reference.
//
//  Usage: kat [--list] [name-substring ...]; exit status 0 iff every selected
//  test passed.  Driven by tests/test_oracle_kat.py.
// =============================================================================
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "lkf_oracle.h"
#include "srtp_oracle.h"

using namespace orc;

namespace {

struct Case {
  const char *name;
  void (*fn)();
};
std::vector<Case> &registry() {
  static std::vector<Case> r;
  return r;
}
struct Reg {
  Reg(const char *n, void (*f)()) { registry().push_back({n, f}); }
};
int g_fail = 0;
const char *g_cur = "";

#define KAT(name)                       \
  static void kat_##name();             \
  static Reg reg_##name(#name, kat_##name); \
  static void kat_##name()

template <typename A, typename B>
void check_eq(const A &a, const B &b, const char *ea, const char *eb, int line) {
  if (!(a == static_cast<A>(b))) {
    g_fail++;
    fprintf(stderr, "  [%s] line %d: %s != %s (%llu vs %llu)\n", g_cur, line, ea, eb,
            (unsigned long long)a, (unsigned long long)static_cast<A>(b));
  }
}
#define EQ(a, b) check_eq((a), (b), #a, #b, __LINE__)
#define TRUE(c) check_eq(bool(c), true, #c, "true", __LINE__)
#define FALSE(c) check_eq(bool(c), false, #c, "false", __LINE__)

void check_bytes(const std::vector<u8> &a, const std::vector<u8> &b, int line) {
  if (a != b) {
    g_fail++;
    fprintf(stderr, "  [%s] line %d: byte vectors differ (len %zu vs %zu):", g_cur, line, a.size(), b.size());
    for (u8 x : a) fprintf(stderr, " %02x", x);
    fprintf(stderr, " |");
    for (u8 x : b) fprintf(stderr, " %02x", x);
    fprintf(stderr, "\n");
  }
}
#define BYTES(a, ...) check_bytes((a), std::vector<u8>(__VA_ARGS__), __LINE__)

// ---------------------------------------------------------------------------
// utils/rangemap_test.go:23-361  TestRangeMapUint32
// ---------------------------------------------------------------------------
using RM32 = RangeMap<u32, u32>;
void expect_ranges(const RM32 &r, std::vector<RM32::RV> want, int line) {
  bool ok = r.ranges.size() == want.size();
  for (size_t i = 0; ok && i < want.size(); i++)
    ok = r.ranges[i].start == want[i].start && r.ranges[i].end == want[i].end && r.ranges[i].value == want[i].value;
  if (!ok) {
    g_fail++;
    fprintf(stderr, "  [%s] line %d: ranges differ; got", g_cur, line);
    for (auto &x : r.ranges) fprintf(stderr, " {%u,%u,%u}", x.start, x.end, x.value);
    fprintf(stderr, "\n");
  }
}
#define RANGES(r, ...) expect_ranges((r), __VA_ARGS__, __LINE__)
u32 rget(const RM32 &r, u32 key, Err want) {
  u32 v = 0;
  Err e = r.GetValue(key, v);
  if (e != want) {
    g_fail++;
    fprintf(stderr, "  [%s] GetValue(%u): err %d, want %d\n", g_cur, key, e, want);
  }
  return v;
}

KAT(rangemap_uint32) {
  RM32 r(2);
  EQ(rget(r, 33333, OK), 0u);
  RANGES(r, {{0, 0, 0}});
  EQ(r.ExcludeRange(10, 11), OK);
  RANGES(r, {{0, 9, 0}, {11, 0, 1}});
  EQ(rget(r, 6, OK), 0u);
  EQ(rget(r, 11, OK), 1u);
  rget(r, 10, ErrKeyExcluded);
  EQ(r.ExcludeRange(9, 10), ErrReversedOrder);
  EQ(r.ExcludeRange(12, 11), ErrReversedOrder);
  EQ(r.ExcludeRange(11, 11), ErrReversedOrder);
  EQ(r.ExcludeRange(11, 12), OK);
  RANGES(r, {{0, 9, 0}, {12, 0, 2}});
  rget(r, 11, ErrKeyExcluded);
  rget(r, 6, OK);
  EQ(rget(r, 12, OK), 2u);
  EQ(r.ExcludeRange(12, 22), OK);
  RANGES(r, {{0, 9, 0}, {22, 0, 12}});
  rget(r, 15, ErrKeyExcluded);
  EQ(rget(r, 25, OK), 12u);
  EQ(r.ExcludeRange(26, 30), OK);
  RANGES(r, {{0, 9, 0}, {22, 25, 12}, {30, 0, 16}});
  EQ(rget(r, 23, OK), 12u);
  EQ(r.ExcludeRange(50, 51), OK);
  RANGES(r, {{22, 25, 12}, {30, 49, 16}, {51, 0, 17}});
  rget(r, 50, ErrKeyExcluded);
  rget(r, 28, ErrKeyExcluded);
  rget(r, 17, ErrKeyTooOld);
  rget(r, 5, ErrKeyTooOld);
  EQ(rget(r, 24, OK), 12u);
  EQ(rget(r, 34, OK), 16u);
  EQ(rget(r, 49, OK), 16u);
  EQ(rget(r, 55555555, OK), 17u);
  r.ClearAndResetValue(24, 23);
  RANGES(r, {{24, 0, 23}});
  EQ(rget(r, 55555555, OK), 23u);
  r.DecValue(34, 12);
  RANGES(r, {{24, 34, 23}, {35, 0, 11}});
  EQ(rget(r, 55555555, OK), 11u);
  EQ(r.ExcludeRange(40, 45), OK);
  RANGES(r, {{24, 34, 23}, {35, 39, 11}, {45, 0, 16}});
  rget(r, 5, ErrKeyTooOld);
  EQ(rget(r, 25, OK), 23u);
  EQ(rget(r, 35, OK), 11u);
  EQ(rget(r, 55555555, OK), 16u);
  r.DecValue(66, 6);
  RANGES(r, {{35, 39, 11}, {45, 66, 16}, {67, 0, 10}});
  rget(r, 25, ErrKeyTooOld);
  EQ(rget(r, 66, OK), 16u);
  EQ(rget(r, 67, OK), 10u);
  r.DecValue(66, 6);
  RANGES(r, {{35, 39, 11}, {45, 66, 16}, {67, 0, 4}});
  EQ(rget(r, 67, OK), 4u);
}

// ---------------------------------------------------------------------------
// utils/wraparound_test.go
// ---------------------------------------------------------------------------
template <typename T, typename ET>
struct WStep {
  T input;
  bool unhandled, restart;
  ET preStart, preHighest, extVal;
  T start;
  ET extStart;
  T highest;
  ET extHighest;
};
template <typename T, typename ET>
void run_wsteps(WrapAround<T, ET> &w, const std::vector<WStep<T, ET>> &steps, int line) {
  int i = 0;
  for (auto &s : steps) {
    auto r = w.Update(s.input);
    bool ok = r.IsUnhandled == s.unhandled && r.IsRestart == s.restart && r.PreExtendedStart == s.preStart &&
              r.PreExtendedHighest == s.preHighest && r.ExtendedVal == s.extVal && w.GetStart() == s.start &&
              w.GetExtendedStart() == s.extStart && w.GetHighest() == s.highest &&
              w.GetExtendedHighest() == s.extHighest;
    if (!ok) {
      g_fail++;
      fprintf(stderr, "  [%s] line %d step %d (input %llu): got u=%d r=%d ps=%llu ph=%llu ev=%llu s=%llu es=%llu h=%llu eh=%llu\n",
              g_cur, line, i, (unsigned long long)s.input, r.IsUnhandled, r.IsRestart,
              (unsigned long long)r.PreExtendedStart, (unsigned long long)r.PreExtendedHighest,
              (unsigned long long)r.ExtendedVal, (unsigned long long)w.GetStart(),
              (unsigned long long)w.GetExtendedStart(), (unsigned long long)w.GetHighest(),
              (unsigned long long)w.GetExtendedHighest());
    }
    i++;
  }
}

// wraparound_test.go:23-195
KAT(wraparound_uint16) {
  const u32 R = 1u << 16, H = 1u << 15;
  WrapAround<u16, u32> w(true);
  run_wsteps<u16, u32>(w,
                       {
                           {10, false, false, 0, 9, 10, 10, 10, 10, 10},
                           {8, false, true, 10, 10, 8, 8, 8, 10, 10},
                           {u16(R - 6), false, true, R + 8, R + 10, R - 6, u16(R - 6), R - 6, 10, R + 10},
                           {u16(R - 12), false, true, R - 6, R + 10, R - 12, u16(R - 12), R - 12, 10, R + 10},
                           {u16(R - 3), false, false, 0, R + 10, R - 3, u16(R - 12), R - 12, 10, R + 10},
                           {10, false, false, 0, R + 10, R + 10, u16(R - 12), R - 12, 10, R + 10},
                           {u16(H - 10), false, false, 0, R + 10, R + H - 10, u16(R - 12), R - 12, u16(H - 10),
                            R + H - 10},
                           {u16(H - 11), false, false, 0, R + H - 10, R + H - 11, u16(R - 12), R - 12, u16(H - 10),
                            R + H - 10},
                           {u16(R - 1), false, false, 0, R + H - 10, R - 1, u16(R - 12), R - 12, u16(H - 10),
                            R + H - 10},
                           {u16(H + 3), false, false, 0, R + H - 10, R + H + 3, u16(R - 12), R - 12, u16(H + 3),
                            R + H + 3},
                       },
                       __LINE__);
}

// wraparound_test.go:197-330
KAT(wraparound_uint16_no_restart) {
  const u32 R = 1u << 16, H = 1u << 15;
  WrapAround<u16, u32> w(false);
  run_wsteps<u16, u32>(w,
                       {
                           {10, false, false, 0, 9, 10, 10, 10, 10, 10},
                           {8, true, false, 0, 10, 8, 10, 10, 10, 10},
                           {u16(R - 6), true, false, 0, 10, R - 6, 10, 10, 10, 10},
                           {u16(R - 12), true, false, 0, 10, R - 12, 10, 10, 10, 10},
                           {10, false, false, 0, 10, 10, 10, 10, 10, 10},
                           {u16(H - 10), false, false, 0, 10, H - 10, 10, 10, u16(H - 10), H - 10},
                           {u16(H + 13), false, false, 0, H - 10, H + 13, 10, 10, u16(H + 13), H + 13},
                           {u16(H - 11), false, false, 0, H + 13, H - 11, 10, 10, u16(H + 13), H + 13},
                       },
                       __LINE__);
}

// wraparound_test.go:332-403
KAT(wraparound_uint16_rollback_restart_reset_highest) {
  WrapAround<u16, u64> w(true);
  w.Update(23);
  EQ(w.GetStart(), 23);
  EQ(w.GetExtendedStart(), 23);
  EQ(w.GetHighest(), 23);
  EQ(w.GetExtendedHighest(), 23);
  w.Update(25);
  EQ(w.GetStart(), 23);
  EQ(w.GetHighest(), 25);
  EQ(w.GetExtendedHighest(), 25);
  auto res = w.Update(12);
  TRUE(res.IsRestart);
  FALSE(res.IsUnhandled);
  EQ(res.PreExtendedStart, 23);
  EQ(res.PreExtendedHighest, 25);
  EQ(res.ExtendedVal, 12);
  EQ(w.GetStart(), 12);
  EQ(w.GetExtendedStart(), 12);
  EQ(w.GetHighest(), 25);
  EQ(w.GetExtendedHighest(), 25);
  w.RollbackRestart(res.PreExtendedStart);
  EQ(w.GetStart(), 23);
  EQ(w.GetExtendedStart(), 23);
  EQ(w.GetHighest(), 25);
  EQ(w.GetExtendedHighest(), 25);
  res = w.Update(65533);
  TRUE(res.IsRestart);
  EQ(res.PreExtendedStart, (1ull << 16) + 23);
  EQ(res.PreExtendedHighest, (1ull << 16) + 25);
  EQ(res.ExtendedVal, 65533);
  EQ(w.GetStart(), 65533);
  EQ(w.GetExtendedStart(), 65533);
  EQ(w.GetHighest(), 25);
  EQ(w.GetExtendedHighest(), 65536 + 25);
  w.RollbackRestart(res.PreExtendedStart);
  EQ(w.GetStart(), 23);
  EQ(w.GetExtendedStart(), 23);
  EQ(w.GetHighest(), 25);
  EQ(w.GetExtendedHighest(), 25);
  w.ResetHighest(0x1234);
  EQ(w.GetStart(), 23);
  EQ(w.GetHighest(), 0x1234);
  EQ(w.GetExtendedHighest(), 0x1234);
  w.ResetHighest(0x7f1234);
  EQ(w.GetStart(), 23);
  EQ(w.GetExtendedStart(), 23);
  EQ(w.GetHighest(), 0x1234);
  EQ(w.GetExtendedHighest(), 0x7f1234);
}

// wraparound_test.go:405-449
KAT(wraparound_uint16_restart_duplicate) {
  WrapAround<u16, u64> w(true);
  w.Update(65534);
  EQ(w.GetStart(), 65534);
  EQ(w.GetExtendedHighest(), 65534);
  w.Update(32);
  EQ(w.GetStart(), 65534);
  EQ(w.GetHighest(), 32);
  EQ(w.GetExtendedHighest(), 65568);
  for (int rep = 0; rep < 2; rep++) {
    auto res = w.Update(65534);
    FALSE(res.IsRestart);
    EQ(res.PreExtendedStart, 0);
    EQ(res.PreExtendedHighest, 65568);
    EQ(res.ExtendedVal, 65534);
    EQ(w.GetStart(), 65534);
    EQ(w.GetExtendedStart(), 65534);
    EQ(w.GetHighest(), 32);
    EQ(w.GetExtendedHighest(), 65568);
  }
}

// wraparound_test.go:451-593
KAT(wraparound_uint32) {
  const u64 R = 1ull << 32, H = 1ull << 31;
  WrapAround<u32, u64> w(true);
  run_wsteps<u32, u64>(w,
                       {
                           {10, false, false, 0, 9, 10, 10, 10, 10, 10},
                           {8, false, true, 10, 10, 8, 8, 8, 10, 10},
                           {u32(R - 6), false, true, R + 8, R + 10, R - 6, u32(R - 6), R - 6, 10, R + 10},
                           {u32(R - 12), false, true, R - 6, R + 10, R - 12, u32(R - 12), R - 12, 10, R + 10},
                           {10, false, false, 0, R + 10, R + 10, u32(R - 12), R - 12, 10, R + 10},
                           {u32(H), false, false, 0, R + 10, R + H, u32(R - 12), R - 12, u32(H), R + H},
                           {u32(H - 1), false, false, 0, R + H, R + H - 1, u32(R - 12), R - 12, u32(H), R + H},
                           {u32(H + 3), false, false, 0, R + H, R + H + 3, u32(R - 12), R - 12, u32(H + 3), R + H + 3},
                       },
                       __LINE__);
}

}  // namespace

// KATs defined in other translation units register themselves the same way.
#include "kat_sfu.inc"
#include "kat_dd.inc"
#include "kat_ddsel.inc"
#include "kat_srtp.inc"
#include "kat_red.inc"
#include "kat_tracker.inc"
#include "kat_nack.inc"
#include "kat_bucket.inc"

int main(int argc, char **argv) {
  bool list = false;
  std::vector<std::string> filt;
  for (int i = 1; i < argc; i++) {
    if (!strcmp(argv[i], "--list"))
      list = true;
    else
      filt.push_back(argv[i]);
  }
  int ran = 0, failed = 0;
  for (auto &c : registry()) {
    if (list) {
      printf("%s\n", c.name);
      continue;
    }
    bool sel = filt.empty();
    for (auto &f : filt)
      if (std::string(c.name).find(f) != std::string::npos) sel = true;
    if (!sel) continue;
    g_cur = c.name;
    int before = g_fail;
    c.fn();
    ran++;
    bool ok = g_fail == before;
    if (!ok) failed++;
    printf("%s %s\n", ok ? "PASS" : "FAIL", c.name);
  }
  if (!list) printf("%d run, %d failed\n", ran, failed);
  return failed ? 1 : 0;
}
