// Exhaustive check that the per-byte UTF-8 rule (snf4j_amd/csrc/ws_rules.h) flags
// exactly the byte at which the reference DFA (Utf8.java, restated in the oracle)
// reaches REJECT, and that utf8_incomplete() equals "final state != ACCEPT".
// Usage: utf8_rule_check <max_len> <n_random>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../snf4j_amd/csrc/ws_rules.h"
extern "C" {
#include "../../oracle/ws_oracle.h"
}

static int64_t rule_first(const uint8_t* s, int n) {
  for (int i = 0; i < n; ++i) {
    uint32_t p1 = i >= 1 ? s[i - 1] : 0, p2 = i >= 2 ? s[i - 2] : 0, p3 = i >= 3 ? s[i - 3] : 0;
    if (ws::utf8_err_byte(p3, p2, p1, s[i])) return i;
  }
  return -1;
}

// word form over a padded buffer: flags for every position, first one wins
static int64_t rule_first_words(const uint8_t* s, int n) {
  std::vector<uint8_t> b(8 + ((n + 3) & ~3) + 4, 0);
  for (int i = 0; i < n; ++i) b[8 + i] = s[i];
  for (int wi = 0; wi * 4 < n; ++wi) {
    uint32_t w, p;
    memcpy(&w, &b[8 + 4 * wi], 4);
    memcpy(&p, &b[4 + 4 * wi], 4);
    uint32_t e = ws::utf8_err_word(w, p);
    for (int j = 0; j < 4 && 4 * wi + j < n; ++j)
      if (e & (0x80u << (8 * j))) return 4 * wi + j;
  }
  return -1;
}

// the kernels' fast rule on a continuation frame: word form over the string, head
// (first 3 bytes) by the exact rule as k_seams does, plus the last-byte test;
// returns the first flag.
static int64_t fast_first(const uint8_t* s, int n) {
  std::vector<uint8_t> b(8 + ((n + 3) & ~3) + 4, 0);
  for (int i = 0; i < n; ++i) b[8 + i] = s[i];
  int64_t first = -1;
  for (int i = 0; i < n && i < 3; ++i) {
    uint32_t p1 = i >= 1 ? s[i - 1] : 0, p2 = i >= 2 ? s[i - 2] : 0, p3 = i >= 3 ? s[i - 3] : 0;
    if (ws::utf8_err_byte(p3, p2, p1, s[i])) return i;
  }
  for (int wi = 0; wi * 4 < n; ++wi) {
    uint32_t w, p;
    memcpy(&w, &b[8 + 4 * wi], 4);
    memcpy(&p, &b[4 + 4 * wi], 4);
    uint32_t e = ws::utf8_err_word_fast(w, p);
    for (int j = 0; j < 4 && 4 * wi + j < n; ++j)
      if (4 * wi + j >= 3 && (e & (0x80u << (8 * j)))) { first = 4 * wi + j; goto done; }
  }
done:
  if (n > 0 && ws::utf8_bad_last(s[n - 1]) && (first < 0 || first > n - 1)) first = n - 1;
  return first;
}

// the kernels' per-word form (U8W: shared shifts, 64-bit pair shifts) must equal
// utf8_err_word_fast in bit 7 of every byte, single words and pairs alike
static long u8w_fails = 0;
static void u8w_check(uint32_t w, uint32_t p) {
  ws::U8W x, q, a, b;
  ws::u8w_one(w, x);
  ws::u8w_one(p, q);
  ws::u8w_pair(p, w, a, b);
  const uint32_t want = ws::utf8_err_word_fast(w, p);
  if ((ws::u8w_err(x, q) & ws::H80) != want || (ws::u8w_err(b, a) & ws::H80) != want) ++u8w_fails;
}

// the fast rule on a message start (a TEXT frame, k_pieces alone): word form over
// the whole string with a zero word before it, plus the last-byte test.
static int64_t fast_first_start(const uint8_t* s, int n) {
  std::vector<uint8_t> b(8 + ((n + 3) & ~3) + 4, 0);
  for (int i = 0; i < n; ++i) b[8 + i] = s[i];
  int64_t first = -1;
  for (int wi = 0; wi * 4 < n && first < 0; ++wi) {
    uint32_t w, p;
    memcpy(&w, &b[8 + 4 * wi], 4);
    memcpy(&p, &b[4 + 4 * wi], 4);
    uint32_t e = ws::utf8_err_word_fast(w, p);
    u8w_check(w, p);
    for (int j = 0; j < 4 && 4 * wi + j < n; ++j)
      if (e & (0x80u << (8 * j))) { first = 4 * wi + j; break; }
  }
  if (n > 0 && ws::utf8_bad_last(s[n - 1]) && (first < 0 || first > n - 1)) first = n - 1;
  return first;
}

static long fails = 0;
static void check(const uint8_t* s, int n) {
  int64_t dfa = or_utf8_reject_pos(0, s, n);
  int64_t r1 = rule_first(s, n), r2 = rule_first_words(s, n), r3 = fast_first(s, n),
          r4 = fast_first_start(s, n);
  bool bad = dfa != r1 || dfa != r2;
  // fast rule: same verdict; first flag at the reject byte, or one byte later when
  // the reject byte is a lead rejected on its own (C0, C1, F5..FF)
  for (int64_t r : {r3, r4}) {
    if (dfa < 0) bad |= r >= 0;
    else bad |= !(r == dfa || (r == dfa + 1 && ws::utf8_bad_last(s[dfa])) || (r == n - 1 && dfa == n - 1));
  }
  if (!bad && dfa < 0) {
    or_utf8_ctx c = {0, 0};
    or_utf8_validate(&c, s, n);
    uint32_t l1 = n >= 1 ? s[n - 1] : 0, l2 = n >= 2 ? s[n - 2] : 0, l3 = n >= 3 ? s[n - 3] : 0;
    bad = (c.state != 0) != ws::utf8_incomplete(l3, l2, l1);
  }
  if (bad && fails++ < 10) {
    printf("MISMATCH dfa=%lld rule=%lld words=%lld fast=%lld start=%lld :", (long long)dfa, (long long)r1,
           (long long)r2, (long long)r3, (long long)r4);
    for (int i = 0; i < n; ++i) printf(" %02x", s[i]);
    printf("\n");
  }
}

int main(int argc, char** argv) {
  int max_len = argc > 1 ? atoi(argv[1]) : 5;
  long n_random = argc > 2 ? atol(argv[2]) : 1000000;
  // every DFA class and every range boundary of the rule
  const uint8_t A[] = {0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2, 0xDF,
                       0xE0, 0xE1, 0xEC, 0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF3, 0xF4, 0xF5, 0xFF};
  const int na = sizeof(A);
  long count = 0;
  for (int n = 1; n <= max_len; ++n) {
    std::vector<int> idx(n, 0);
    std::vector<uint8_t> s(n);
    for (;;) {
      for (int i = 0; i < n; ++i) s[i] = A[idx[i]];
      check(s.data(), n);
      ++count;
      int i = n - 1;
      while (i >= 0 && ++idx[i] == na) idx[i--] = 0;
      if (i < 0) break;
    }
  }
  // all 2-byte strings over the full byte range, then random strings
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b) { uint8_t s[2] = {(uint8_t)a, (uint8_t)b}; check(s, 2); ++count; }
  uint64_t x = 12345;
  for (long r = 0; r < n_random; ++r) {
    uint8_t s[64];
    int n = 1 + (int)(or_splitmix64(x++) % 64);
    for (int i = 0; i < n; ++i) {
      uint64_t v = or_splitmix64(x++);
      s[i] = (v & 3) == 0 ? (uint8_t)(v >> 8) : A[(v >> 8) % na];
    }
    check(s, n);
    ++count;
  }
  // every (previous byte, byte) pair at every byte position of the word
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b)
      for (int j = 0; j < 4; ++j) {
        const uint64_t v = ((uint64_t)b << 32 | (uint64_t)a << 24) << (8 * j);
        u8w_check((uint32_t)(v >> 32), (uint32_t)v);
      }
  printf("checked %ld strings, %ld mismatches, %ld per-word form mismatches\n", count, fails, u8w_fails);
  return fails || u8w_fails ? 1 : 0;
}
