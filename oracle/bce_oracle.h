/*
 * bce_oracle.h -- CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This is the CHECKER, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load liboracle.so.  The shipped engine
 * (bayesian-consensus-engine_amd/) never links or imports it.
 *
 * Every function is a scalar, sequential restatement of the reference Python
 * (consensus-nexus/bayesian-consensus-engine, src/bayesian_engine/), compiled with
 * -ffp-contract=off so every float op rounds exactly like CPython's.  It is pinned
 * bit-for-bit against golden vectors captured from the reference itself
 * (tests/golden/gen_golden.py, tests/test_oracle_golden.py).
 *
 * Layout conventions (shared with include/bce.h):
 *   CSR markets: offsets[M+1] int64, sid[N] int32 (interned rank ids: integer order ==
 *   Python str order), prob[N] fp64.  Source table: rel[S], conf[S] fp64 with the
 *   cold-start defaults already baked in, present[S] u8 (key present in the dict).
 *   Per-unique outputs sit at the market's CSR offsets: slot offsets[m]+j, j < n_unique[m].
 *   usid carries the cold bit in bit 31.
 */
#ifndef BCE_ORACLE_H
#define BCE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_NO_TIMESTAMP INT64_MIN

/* core.compute_consensus over CSR (core.py:63-179) + range validation (core.py:59-60).
 * consensus is 0.0 where null (null <=> total_weight == 0, or empty market). */
int orc_consensus_csr(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                      const double* prob, const double* rel, const double* conf,
                      const uint8_t* present, int32_t n_sources, double* consensus,
                      double* confidence, double* total_weight, int32_t* n_unique,
                      int32_t* err_idx, int32_t* usid, double* weight, double* nweight);

/* decay.compute_decay_factor (decay.py:31-58) */
double orc_decay_factor(double elapsed_days, double half_life_days);
/* decay.apply_reliability_decay (decay.py:61-100) */
double orc_apply_decay(double r, double elapsed_days, double half_life_days, double min_rel);
/* decay.days_since_update for int64 microsecond stamps (decay.py:103-145) */
double orc_days_since(int64_t now_us, int64_t t_us);

/* get_reliability(apply_decay=True) over a whole table (reliability.py:110-140) */
void orc_decay_view(int64_t n, const double* rel, const int64_t* t_us, const uint8_t* present,
                    int64_t now_us, double half_life_days, double min_rel, double default_rel,
                    double* view);

/* compute_update / update_reliability math (reliability.py:142-183), one outcome per
 * source: flags bit0 = participates, bit1 = correct.  Absent rows start cold. */
void orc_outcome_update(int64_t n, double* rel, double* conf, int64_t* t_us, uint8_t* present,
                        const uint8_t* flags, int64_t now_us, double default_rel,
                        double default_conf);

/* CrossMarketAggregator.summarize_sources counts (market.py:277-319).
 * outcome[m]: -1 unresolved / skipped, 0 false, 1 true.  Counts are added. */
void orc_agreement_stats(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                         const double* prob, const int8_t* outcome, int32_t* correct,
                         int32_t* total);

/* Python round(x, 6) (tiebreak.py:54) */
double orc_round_decimal(double x, int ndigits);

/* DeterministicTieBreaker.resolve over CSR markets (tiebreak.py:73-152).
 * Per market: winner, label (0 unanimous, 1 weight_density, 2 prediction_value_smallest,
 * 3 single_agent), n_groups, variance; per group (at CSR offsets, first-seen order):
 * key, count, total_weight, avg_conf, max_rel.  Empty market: n_groups = -1. */
int orc_tiebreak_csr(const int64_t* offsets, int64_t n_markets, const double* pred,
                     const double* conf, const double* weight, const double* rel,
                     const double* keys,
                     double* winner, int32_t* label, int32_t* n_groups, double* variance,
                     double* g_key, int32_t* g_count, double* g_total, double* g_avgconf,
                     double* g_maxrel);

/* Config-5 re-estimation (composition of core.py:130-144 and market.py:298-310):
 * P is [A][M] row-major (agent-major).  iters passes; w in/out [A]; per pass the
 * consensus of every market (sorted-agent order), then agreement counts and
 * w_a = correct/total.  cons_out [iters][M] (0.0 where null), null_out, agree_out [iters][A]. */
void orc_reestimate(const double* P, int64_t A, int64_t M, int iters, double* w,
                    double* cons_out, uint8_t* null_out, int64_t* agree_out);

/* NamespacedReliabilityStore.get_reliability (reliability_abstraction.py:119-188) over
 * a rank space: three scopes (market, domain, global), NULL rel = not requested. */
void orc_namespace_resolve(int64_t n, const double* const rel[3], const double* const conf[3],
                           const int64_t* const t_us[3], const uint8_t* const has[3],
                           int apply_decay, int64_t now_us, double half_life_days, double min_rel,
                           double default_rel, double default_conf, double* rel_out,
                           double* conf_out, uint8_t* scope_out);

/* CrossMarketAggregator.aggregate_consensus (market.py:340-408) per member group. */
void orc_aggregate_groups(const int64_t* goff, int64_t n_groups, const int64_t* members,
                          const double* cons, const double* conf, const uint8_t* has,
                          double* wavg, double* median, double* majority, double* mean_conf,
                          int64_t* n_included);

#ifdef __cplusplus
}
#endif
#endif
