/* oracle_fuzz.c -- sanitizer harness for the CPU restatement (oracle/bce_oracle.c), CPU only.
 *
 * Built by `make -C oracle asan` with -fsanitize=address,undefined (tests/test_sanitizers.py
 * runs it).  Random batches over every entry point: ragged CSR with empty markets, long
 * markets, duplicate and hot sources, NaN / out-of-range probabilities; tie-breaks with grid
 * and signed-zero predictions; decay / update over absent rows and NO_TIMESTAMP stamps; the
 * namespaced fallback with missing scopes; aggregation with empty groups; a small
 * re-estimation.  Memory errors and UB are the sanitizers' to report. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/bce_oracle.h"

static uint64_t g_s = 88172645463325252ull;
static uint64_t rnd(void) { g_s ^= g_s << 13; g_s ^= g_s >> 7; g_s ^= g_s << 17; return g_s; }
static double urand(void) { return (double)(rnd() >> 11) * (1.0 / 9007199254740992.0); }

static void* xcalloc(size_t n, size_t sz) {
  void* p = calloc(n ? n : 1, sz);
  if (!p) { fprintf(stderr, "oracle_fuzz: out of memory\n"); exit(2); }
  return p;
}

static void one_batch(int it) {
  const int64_t M = 1 + (int64_t)(rnd() % 300);
  const int32_t S = 1 + (int32_t)(rnd() % 500);
  int64_t* off = xcalloc(M + 1, sizeof *off);
  for (int64_t m = 0; m < M; ++m) {
    const uint64_t r = rnd() % 100;
    const int64_t n = r < 10 ? 0 : r < 80 ? (int64_t)(rnd() % 40) : r < 98 ? (int64_t)(rnd() % 700) : 5000;
    off[m + 1] = off[m] + n;
  }
  const int64_t N = off[M];
  int32_t* sid = xcalloc(N, sizeof *sid);
  double *prob = xcalloc(N, sizeof *prob), *conf_s = xcalloc(N, sizeof *conf_s), *w = xcalloc(N, sizeof *w);
  double *rel_s = xcalloc(N, sizeof *rel_s), *keys = xcalloc(N, sizeof *keys);
  for (int64_t i = 0; i < N; ++i) {
    sid[i] = (rnd() % 4) ? (int32_t)(rnd() % S) : (int32_t)(rnd() % (S < 4 ? S : 4));
    const uint64_t k = rnd() % 50;
    prob[i] = k == 0 ? NAN : k == 1 ? 1.5 : k == 2 ? -0.0 : k < 10 ? (double)(rnd() % 10) / 10.0 : urand();
    conf_s[i] = urand();
    w[i] = (rnd() % 3) ? urand() : 0.0;
    rel_s[i] = urand();
    keys[i] = orc_round_decimal(prob[i], 6);
  }
  double *rel = xcalloc(S, sizeof *rel), *conf = xcalloc(S, sizeof *conf);
  uint8_t* present = xcalloc(S, 1);
  for (int32_t s = 0; s < S; ++s) {
    present[s] = (rnd() % 10) != 0;
    rel[s] = present[s] ? urand() : 0.5;
    conf[s] = present[s] ? urand() : 0.25;
  }
  double *cons = xcalloc(M, 8), *cf = xcalloc(M, 8), *tot = xcalloc(M, 8), *wt = xcalloc(N, 8), *nw = xcalloc(N, 8);
  int32_t *nu = xcalloc(M, 4), *ei = xcalloc(M, 4), *us = xcalloc(N, 4);
  orc_consensus_csr(off, M, sid, prob, rel, conf, present, S, cons, cf, tot, nu, ei, us, wt, nw);
  double *win = xcalloc(M, 8), *var = xcalloc(M, 8), *gk = xcalloc(N, 8), *gt = xcalloc(N, 8), *ga = xcalloc(N, 8),
         *gm = xcalloc(N, 8);
  int32_t *lab = xcalloc(M, 4), *ng = xcalloc(M, 4), *gc = xcalloc(N, 4);
  orc_tiebreak_csr(off, M, prob, conf_s, w, rel_s, keys, win, lab, ng, var, gk, gc, gt, ga, gm);
  int8_t* outcome = xcalloc(M, 1);
  for (int64_t m = 0; m < M; ++m) outcome[m] = (int8_t)((int)(rnd() % 3) - 1);
  int32_t *correct = xcalloc(S, 4), *total = xcalloc(S, 4);
  orc_agreement_stats(off, M, sid, prob, outcome, correct, total);
  /* decay / outcome update over the table */
  int64_t* t_us = xcalloc(S, 8);
  uint8_t* flags = xcalloc(S, 1);
  double* view = xcalloc(S, 8);
  const int64_t now = 1772323200000000ll;
  for (int32_t s = 0; s < S; ++s) {
    t_us[s] = (rnd() % 8) ? now - (int64_t)(urand() * 9e12) : ORC_NO_TIMESTAMP;
    flags[s] = (uint8_t)(rnd() % 4);
  }
  orc_decay_view(S, rel, t_us, present, now, 30.0, 0.1, 0.5, view);
  orc_outcome_update(S, rel, conf, t_us, present, flags, now, 0.5, 0.25);
  /* namespaced fallback: scope 1 missing on odd iterations */
  const double* r3[3] = {rel, (it & 1) ? NULL : conf, view};
  const double* c3[3] = {conf, (it & 1) ? NULL : rel, conf};
  const int64_t* t3[3] = {t_us, (it & 1) ? NULL : t_us, t_us};
  const uint8_t* h3[3] = {present, (it & 1) ? NULL : flags, present};
  double *ro = xcalloc(S, 8), *co = xcalloc(S, 8);
  uint8_t* so = xcalloc(S, 1);
  orc_namespace_resolve(S, r3, c3, t3, h3, it & 2, now, 30.0, 0.1, 0.5, 0.25, ro, co, so);
  /* aggregation: groups of random member lists (some empty) */
  const int64_t G = 1 + (int64_t)(rnd() % 40);
  int64_t* goff = xcalloc(G + 1, 8);
  for (int64_t g = 0; g < G; ++g) goff[g + 1] = goff[g] + (int64_t)(rnd() % 60);
  int64_t* mem = xcalloc(goff[G], 8);
  uint8_t* has = xcalloc(M, 1);
  for (int64_t i = 0; i < goff[G]; ++i) mem[i] = (int64_t)(rnd() % M);
  for (int64_t m = 0; m < M; ++m) has[m] = (rnd() % 5) != 0;
  double *wa = xcalloc(G, 8), *md = xcalloc(G, 8), *mj = xcalloc(G, 8), *mc = xcalloc(G, 8);
  int64_t* inc = xcalloc(G, 8);
  orc_aggregate_groups(goff, G, mem, cons, cf, has, wa, md, mj, mc, inc);
  /* re-estimation on a small dense matrix */
  const int64_t A = 1 + (int64_t)(rnd() % 20), MM = 1 + (int64_t)(rnd() % 50);
  double *P = xcalloc(A * MM, 8), *wr = xcalloc(A, 8), *co2 = xcalloc(2 * MM, 8);
  uint8_t* nl = xcalloc(2 * MM, 1);
  int64_t* ag = xcalloc(2 * A, 8);
  for (int64_t i = 0; i < A * MM; ++i) P[i] = (rnd() % 30) ? urand() : NAN;
  for (int64_t a = 0; a < A; ++a) wr[a] = 0.5;
  orc_reestimate(P, A, MM, 2, wr, co2, nl, ag);
  void* ptrs[] = {off, sid, prob, conf_s, w, rel_s, keys, rel, conf, present, cons, cf, tot, wt, nw, nu, ei, us,
                  win, var, gk, gt, ga, gm, lab, ng, gc, outcome, correct, total, t_us, flags, view, ro, co, so,
                  goff, mem, has, wa, md, mj, mc, inc, P, wr, co2, nl, ag};
  for (size_t i = 0; i < sizeof ptrs / sizeof ptrs[0]; ++i) free(ptrs[i]);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  for (int it = 0; it < iters; ++it) one_batch(it);
  printf("oracle_fuzz ok: %d random batches\n", iters);
  return 0;
}
