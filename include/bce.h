/*
 * bce.h -- C ABI of the MI355X-native batched consensus engine (libbce_hip.so).
 *
 * This is the drop-in boundary for the reference's hot path
 * (consensus-nexus/bayesian-consensus-engine, src/bayesian_engine/).  The reference is
 * pure Python and exposes no plugin registry, so the boundary is
 * this C ABI, bound from Python with ctypes (see INTEGRATION.md for the binding a
 * maintainer of the reference would add).  Every entry point names the reference
 * function it replaces.
 *
 * Conventions
 *  - All arrays are DEVICE pointers (hipMalloc / torch tensors on cuda:N) unless the
 *    name ends in _host.  Work is enqueued on `stream` (a hipStream_t; NULL = the
 *    legacy default stream).  Nothing synchronises unless stated.
 *  - Every entry point returns an int status: BCE_OK (0) or a negative BCE_E*; the
 *    library keeps no global mutable state besides the last-error string
 *    (bce_last_error(), thread-local).  The caller owns every buffer; the library never
 *    frees caller memory.
 *  - Markets are CSR: offsets[M+1] int64 (offsets[0] may be non-zero: a shard view),
 *    sid[N] int32 = interned source rank ids whose integer order equals Python's
 *    sorted() order of the sourceId strings (code-point order), prob[N] fp64.
 *  - The consensus source table is dense over rank ids and laid out for the gather:
 *    relconf[2*S] fp64 = interleaved {reliability, confidence} pairs (16-byte aligned, one
 *    16-B load per unique source) with the cold-start defaults (config.py:17-18) baked in
 *    for absent keys, and present_bits[ceil(S/32)] u32 = bit s%32 of word s/32 set iff
 *    the sourceId is a key of source_reliability (core.py:167-170).  bce_table_pack
 *    builds it from separate rel/conf/present arrays.
 *  - Per-unique-source outputs are written at the market's CSR offsets: slot
 *    offsets[m]+j for j < n_unique[m].  Slots n_unique[m] <= j < n (the market's length)
 *    are scratch: a kernel may leave them untouched or write unspecified values there
 *    (the short-market kernel stores whole 16-byte chunks).  Nothing outside the
 *    market's own [offsets[m], offsets[m+1]) range is ever written.  usid carries the
 *    cold-start bit in bit 31 (value = rank | cold << 31).
 *  - Floating point follows CPython: no fused multiply-add anywhere on the parity path,
 *    sums in the reference's order in BCE_MODE_EXACT (bit-exact vs the reference).
 */
#ifndef BCE_H
#define BCE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BCE_ABI_VERSION 3  /* 3: BCE_NBINS 13 (1536 and 3072 length bins), tie-break per-group scratch slots */

enum bce_status {
    BCE_OK = 0,
    BCE_EINVAL = -1,      /* bad argument (null pointer, size, sid out of range) */
    BCE_EHIP = -2,        /* a HIP runtime call failed (message in bce_last_error) */
    BCE_EUNSUPPORTED = -3 /* shape outside what this build handles */
};

enum bce_mode {
    BCE_MODE_EXACT = 0, /* reference summation order: bit-exact outputs */
    BCE_MODE_FAST = 1   /* tree reductions for long markets (<= 1e-9 abs vs reference) */
};
/* BCE_MODE_FAST reproducibility: deterministic for a given call (the same launch reproduces
 * every bit), but NOT invariant to batch composition.  bce_consensus_planned merges a small
 * call's non-power-of-two bins (1025..1536, 2049..3072) into the launch of the bin above when a
 * launch would fill fewer than 6 rounds of its resident grid (which depends on the market count
 * and the GPU's CU count); the wider workgroup sums the partial totals over 8 instead of 6 (4
 * instead of 3) waves.  So one market's consensus / confidence / total weight / normalizedWeight
 * can differ in the last bits between a full batch, a shard of it, or another GPU model -- always
 * within the 1e-9 bound.  Integer outputs, usid and weight are bit-exact in both modes, and
 * BCE_MODE_EXACT is bit-identical in every launch shape. */

/* Tie-break labels (tiebreak.py:123-133, 89-96). */
enum bce_tb_label {
    BCE_TB_UNANIMOUS = 0,
    BCE_TB_WEIGHT_DENSITY = 1,
    BCE_TB_PREDICTION_VALUE_SMALLEST = 2,
    BCE_TB_SINGLE_AGENT = 3
};

#define BCE_NO_TIMESTAMP INT64_MIN /* falsy / unparseable updated_at (decay.py:125-131) */

/* ---- library ------------------------------------------------------------------ */
int bce_abi_version(void);
const char* bce_last_error(void);
/* Number of visible devices (0 on a machine without a GPU; never fails). */
int bce_device_count(void);
/* Synchronise `stream` and report (then clear) the current device's fault word: a kernel
 * that had to give up -- a persistent wave whose bounded wait expired, a sid >= n_sources,
 * a market longer than the max_len it was launched with -- records a code there instead
 * of failing silently.  BCE_OK when clean, else BCE_EHIP with the reason in
 * bce_last_error(). */
int bce_fault_check(void* stream);
/* Test hook: polls a persistent wave makes before giving up (<= 0 restores the default,
 * 2^22).  A tiny cap makes the pipe kernel's waves give up at once, which exercises the
 * fault path above; results of such a launch are garbage. */
int bce_debug_set_spin_cap(int cap);
/* Self-test of the wide kernel's VALU lane exchanges (DPP / permlane swaps) and wave scan:
 * one wave writes 13*64 words to `out` (see consensus_wide.hip); tests run it first. */
int bce_debug_lane_selftest(unsigned* out, void* stream);
/* Host run of the exact big-integer round(x, ndigits) the tie-break kernels use for
 * 23 <= ndigits <= 323 and -308 <= ndigits <= -16 (valid for any 1 <= |ndigits| in range):
 * for the CPU tests against Python round().  *overflow = 1 where CPython raises
 * OverflowError.  No GPU needed. */
double bce_debug_py_round(double x, int32_t ndigits, int32_t* overflow);

/* ---- consensus: core.compute_consensus (core.py:63-179) + validation -------------
 *
 * Replaces: core.compute_consensus(signals, source_reliability) for every market of
 * the batch, and the numeric part of core.validate_input_payload (core.py:59-60):
 * err_idx[m] = first signal index whose probability is < 0 or > 1 (NaN passes), -1 if
 * none.  Also the batch loop MarketStore.compute_all_consensus (market.py:200-221).
 *
 * Outputs per market: consensus (0.0 where null), confidence, total_weight,
 * n_unique, err_idx (may be NULL to skip).  null <=> total_weight == 0 (core.py:131)
 * or the market is empty (core.py:88-96).  Per unique source (sorted by rank):
 * usid (rank | cold<<31), weight (= reliability, core.py:119), nweight
 * (core.py:151).  Any of usid/weight/nweight may be NULL ("compact" mode).
 *
 * market_list (nullable): process only markets market_list[0..n_list) (ascending
 * market indices recommended).  NULL = all markets 0..n_markets.  max_len is an
 * upper bound on the market lengths processed (0 = unknown: the library computes it,
 * which synchronises the stream).  n_sources bounds sid.
 */
int bce_consensus_csr(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                      const double* prob, int64_t n_signals, const double* relconf,
                      const uint32_t* present_bits, int32_t n_sources,
                      const int32_t* market_list, int64_t n_list, int32_t max_len, int32_t mode,
                      double* consensus, double* confidence, double* total_weight,
                      int32_t* n_unique, int32_t* err_idx, int32_t* usid, double* weight,
                      double* nweight, void* stream);

/* Pack separate rel[S], conf[S], present[S] (u8, nullable = all present) into the
 * consensus table layout: relconf[2*S] interleaved, present_bits[ceil(S/32)]. */
int bce_table_pack(int64_t n, const double* rel, const double* conf, const uint8_t* present,
                   double* relconf, uint32_t* present_bits, void* stream);

/* Validation only (core.validate_input_payload's numeric check, core.py:59-60):
 * err_idx[m] = first signal index with probability < 0 or > 1 (NaN passes), -1 if none.
 * The structural/type checks (core.py:34-58) are done where the Python objects live. */
int bce_validate_csr(const int64_t* offsets, int64_t n_markets, const double* prob,
                     int32_t* err_idx, void* stream);

/* Host-planned variant for ragged batches: the caller bins markets by length once
 * (bce_plan_bins on HOST offsets) and passes the device copy of the ordered market
 * list plus the bin boundaries.  bin_start has BCE_NBINS+1 entries (host array).  Inside
 * a bin markets keep their index order, except the wide bins (65..4096 signals), which
 * are ordered longest first (ties by index) so each launch ends on its short markets.
 * bce_consensus_planned runs the n <= 64 bins on a library-owned side stream (one per
 * device) forked from `stream` by an event and joined back into it before it returns, so
 * the caller sees ordinary stream order; concurrent callers are serialised over the fork. */
#define BCE_NBINS 13 /* n<=8, <=16, <=32, <=64, <=128, <=256, <=512, <=1024, <=1536, <=2048, <=3072, <=4096, >4096 */
int bce_plan_bins(const int64_t* offsets_host, int64_t n_markets, int32_t* order_host,
                  int64_t* bin_start_host, int32_t* max_len_host);
/* The same plan built on the GPU from DEVICE offsets (no D2H copy of the CSR, no host sort):
 * a stable two-pass LSD radix sort of the market indices by a 12-bit key (bin, then longest
 * first inside the wide bins), so `order` (device int32[n_markets]) is bit-identical to
 * bce_plan_bins'.  Enqueued on `stream`; the call then SYNCHRONISES that stream to return the
 * bin boundaries (host int64[BCE_NBINS+1]), the longest market (host, nullable) and the >4096
 * bin's scratch bytes for bce_consensus_planned (host, nullable).  scratch: device buffer of
 * bce_plan_device_scratch_bytes(n_markets) bytes (256-byte aligned).  Decreasing offsets ->
 * BCE_EINVAL (as bce_plan_bins).  Replaces the per-call host planning of a fresh batch
 * (the reference sorts each market's sources, core.py:103, inside its market loop,
 * market.py:200-221). */
int bce_plan_bins_device(const int64_t* offsets, int64_t n_markets, int32_t* order, int64_t* bin_start_host,
                         int32_t* max_len_host, int64_t* long_scratch_bytes_host, void* scratch,
                         int64_t scratch_bytes, void* stream);
int64_t bce_plan_device_scratch_bytes(int64_t n_markets);
/* The same plan without any host synchronisation: the bin boundaries stay on the device
 * (bin_start_dev, device int64[BCE_NBINS+1]); decreasing offsets raise the device fault word
 * (bce_fault_check) and leave every bin empty.  Pair with bce_consensus_planned_device. */
int bce_plan_bins_device_async(const int64_t* offsets, int64_t n_markets, int32_t* order, int64_t* bin_start_dev,
                               void* scratch, int64_t scratch_bytes, void* stream);
/* bce_consensus_planned over a device-resident plan: every bin's kernel reads its range of the
 * plan order on the device, so planning + consensus of a fresh batch enqueue with no host sync.
 * Launch structure of a full batch (no small-call merges).  Markets longer than 4096 signals are
 * not computed and raise the device fault word (use bce_plan_bins_device + bce_consensus_planned
 * for them); n_sources must be <= 2^25. */
int bce_consensus_planned_device(const int64_t* offsets, int64_t n_markets, const int32_t* sid, const double* prob,
                                 int64_t n_signals, const double* relconf, const uint32_t* present_bits,
                                 int32_t n_sources, const int32_t* order, const int64_t* bin_start_dev,
                                 int32_t mode, double* consensus, double* confidence, double* total_weight,
                                 int32_t* n_unique, int32_t* err_idx, int32_t* usid, double* weight,
                                 double* nweight, void* stream);
/* Bytes of device scratch bce_consensus_planned needs for the >4096 bin. */
int64_t bce_consensus_scratch_bytes(const int64_t* offsets_host, const int32_t* order_host,
                                    const int64_t* bin_start_host);
int bce_consensus_planned(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                          const double* prob, int64_t n_signals, const double* relconf,
                          const uint32_t* present_bits, int32_t n_sources,
                          const int32_t* order, const int64_t* bin_start_host, int32_t mode,
                          double* consensus, double* confidence, double* total_weight,
                          int32_t* n_unique, int32_t* err_idx, int32_t* usid, double* weight,
                          double* nweight, void* scratch, int64_t scratch_bytes, void* stream);

/* ---- decay: get_reliability(apply_decay=True) over a table ----------------------
 * Replaces: decay.apply_reliability_decay (decay.py:61-100) composed with
 * decay.days_since_update (decay.py:103-145) as used by
 * SQLiteReliabilityStore.get_reliability (reliability.py:110-131).
 * view[s] = present[s] ? decay(rel[s], days(now_us - t_us[s])) : default_rel.
 * present may be NULL (all present).  t_us[s] == BCE_NO_TIMESTAMP means no decay. */
int bce_decay_view(int64_t n, const double* rel, const int64_t* t_us, const uint8_t* present,
                   int64_t now_us, double half_life_days, double min_rel, double default_rel,
                   double* view, void* stream);

/* ---- decay on elapsed days: decay.compute_decay_factor (decay.py:31-58) and
 * decay.apply_reliability_decay (decay.py:61-100), elementwise.  factor (nullable) gets
 * 2^(-days/h) (1.0 where days <= 0); out (nullable) gets the decayed reliability. */
int bce_decay_apply(int64_t n, const double* rel, const double* elapsed_days,
                    double half_life_days, double min_rel, double* out, double* factor,
                    void* stream);

/* ---- outcome update: compute_update / update_reliability (reliability.py:142-233) --
 * One outcome per source per call: flags[s] bit0 = participates, bit1 = correct.
 * Participants: rel = clamp(rel +- MAX_UPDATE_STEP) (reliability.py:163-169),
 * conf = min(1, conf + (1-conf)*0.1) (:172-173), t_us = now_us (:175), present = 1.
 * Absent rows start from (default_rel, default_conf) (reliability.py:133-140). */
int bce_outcome_update(int64_t n, double* rel, double* conf, int64_t* t_us, uint8_t* present,
                       const uint8_t* flags, int64_t now_us, double default_rel,
                       double default_conf, void* stream);

/* ---- replay step (config 4): decayed view at now_us, then the outcome update --------
 * flags2 is 2-bit packed: source s uses bits 2*(s%4)..+1 of byte s/4 (bit0 participates,
 * bit1 correct).  Equivalent to bce_decay_view followed by bce_outcome_update. */
int bce_replay_step(int64_t n, double* rel, double* conf, int64_t* t_us, uint8_t* present,
                    const uint8_t* flags2, int64_t now_us, double half_life_days,
                    double min_rel, double default_rel, double default_conf, double* view,
                    void* stream);

/* ---- namespaced fallback: NamespacedReliabilityStore.get_reliability ----------------
 * Replaces reliability_abstraction.py:119-188 for every source of a rank space at once.
 * Up to three scope tables in precedence order: scope 0 = market (the row keyed by
 * market_id), 1 = domain ("__domain__:<domain>"), 2 = global ("__global__"); a NULL rel
 * skips the scope, as a falsy market_id / domain does (:136, :150).  has[s] != 0 iff the
 * scope holds a row with a truthy updated_at (the `if record.updated_at:` tests).  The
 * first scope with has[s] supplies (reliability, confidence); the reliability is decayed
 * at now_us when apply_decay, as SQLiteReliabilityStore.get_reliability does
 * (reliability.py:114-123; t_us == BCE_NO_TIMESTAMP = unparseable = no decay).  No scope
 * => the cold-start defaults (:177-186).  Outputs (each nullable, at least one given):
 * relconf[2*n] = the packed consensus table, present_bits = bit set for every source
 * (mark_cold = 0: callers put every sourceId in the dict) or only for sources that
 * resolved to a stored row (mark_cold = 1), scope[s] = 0/1/2, or 3 for cold start. */
int bce_namespace_resolve(int64_t n, const double* rel0, const double* conf0, const int64_t* t0,
                          const uint8_t* has0, const double* rel1, const double* conf1,
                          const int64_t* t1, const uint8_t* has1, const double* rel2,
                          const double* conf2, const int64_t* t2, const uint8_t* has2,
                          int apply_decay, int64_t now_us, double half_life_days, double min_rel,
                          double default_rel, double default_conf, int mark_cold, double* relconf,
                          uint32_t* present_bits, uint8_t* scope, void* stream);

/* ---- tie-break: DeterministicTieBreaker.resolve (tiebreak.py:73-152) per market -----
 * Per signal: pred (AgentSignal.prediction), conf, weight, rel (reliability_score).
 * Per market: winner (rounded group key, or the raw prediction for a single agent),
 * label (enum bce_tb_label; -1 for an empty market = the reference's ValueError),
 * n_groups, variance (unrounded population variance of conf, tiebreak.py:108-110).
 * Per group, first-seen order, at CSR offsets: key, count, weight density, avg conf,
 * max reliability (tiebreak.py:58-71); per signal (nullable g_of) the ordinal of its group,
 * which lets a caller rebuild the reference's dict keys with their Python types (an int
 * prediction keys its group with an int).  Group pointers may be NULL.  ndigits is the
 * DeterministicTieBreaker precision: CPython round(x, ndigits) restated exactly for every
 * int (tiebreak.py:46-47,54): -15 <= ndigits <= 22 with doubles, ndigits < -308 (signed
 * zero), ndigits > 323 (x itself), the rest with exact big integers (py_round_big.hpp).  A
 * rounded key too large for a double (ndigits <= -16, |x| near DBL_MAX: CPython raises
 * OverflowError) sets device fault 6, which bce_fault_check reports.
 * Slots n_groups <= j < n of a market's per-group outputs are scratch (unspecified values).
 * bce_tiebreak_csr: markets market_list[0..n_list) (NULL = all), every length <= max_len
 * <= 64 (one lane per market up to 32 agents, one wave per market beyond).  bce_tiebreak_csr_long: markets of any length >= 1, max_len
 * >= every listed market's length (one workgroup per market; sorted in LDS up to 4096
 * agents, beyond that in a global scratch slice the library allocates on `stream`). */
int bce_tiebreak_csr(const int64_t* offsets, int64_t n_markets, const int32_t* market_list,
                     int64_t n_list, const double* pred, const double* conf, const double* weight,
                     const double* rel, int32_t max_len, int32_t ndigits, double* winner,
                     int32_t* label, int32_t* n_groups, double* variance, double* g_key,
                     int32_t* g_count, double* g_density, double* g_avgconf, double* g_maxrel,
                     int32_t* g_of, void* stream);
int bce_tiebreak_csr_long(const int64_t* offsets, int64_t n_markets, const int32_t* list,
                          int64_t n_list, int32_t ndigits, const double* pred, const double* conf,
                          const double* weight, const double* rel, int64_t max_len, double* winner,
                          int32_t* label, int32_t* n_groups, double* variance, double* g_key,
                          int32_t* g_count, double* g_density, double* g_avgconf, double* g_maxrel,
                          int32_t* g_of, void* stream);

/* ---- agreement statistics: CrossMarketAggregator.summarize_sources counts -----------
 * (market.py:279-304).  outcome[m]: -1 skip (unresolved), 0 false, 1 true.
 * correct[sid] / total[sid] are ACCUMULATED (zero them first); int32 atomics, exact. */
int bce_agreement_stats(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                        const double* prob, const int8_t* outcome, int32_t* correct,
                        int32_t* total, void* stream);

/* ---- cross-market aggregation: CrossMarketAggregator.aggregate_consensus ------------
 * (market.py:340-408) for n_groups groups at once.  Group g is the ordered member list
 * members[group_offsets[g] .. group_offsets[g+1]) of market indices (< n_markets; the
 * markets matched by the patterns in list_markets order, duplicates kept, :355-357).
 * has_consensus[m] != 0 iff market m has a consensus result whose consensus is not None
 * (:369-375).  Per group (outputs nullable): wavg = weighted_average (:386-393), median
 * = sorted(consensus)[k // 2] (:394-397), majority (:398-401), mean_conf = the result's
 * confidence (:407), n_included = k.  k == 0 => the float outputs are NaN (the reference
 * returns consensus None).  Sums are left to right in list order: bit-exact. */
int bce_aggregate_groups(const int64_t* group_offsets, int64_t n_groups, const int64_t* members,
                         int64_t n_markets, const double* consensus, const double* confidence,
                         const uint8_t* has_consensus, double* wavg, double* median,
                         double* majority, double* mean_conf, int64_t* n_included, void* stream);

/* ---- re-estimation (config 5): consensus <-> reliability over a dense matrix --------
 * P is agent-major [A][ld] fp64 (column m of market m; ld >= M).  One pass:
 *   consensus[m] = sum_a P[a][m]*w[a] / sum_a w[a]  (agent order, core.py:130-144),
 *   null[m] = (sum_a w[a] == 0);
 * then agreement[a] += #{m not null : (P[a][m] >= 0.5) == (consensus[m] >= 0.5)}
 * (market.py:298-304) and resolved += #{m not null}.  w_new[a] = agree/resolved
 * (0.5 if resolved == 0, market.py:310) is bce_reestimate_weights. */
int bce_reestimate_consensus(const double* P, int64_t A, int64_t M, int64_t ld, const double* w,
                             double* consensus, uint8_t* null_out, void* stream);
int bce_reestimate_agreement(const double* P, int64_t A, int64_t M, int64_t ld,
                             const double* consensus, const uint8_t* null_in,
                             int64_t* agreement, int64_t* resolved, void* stream);
int bce_reestimate_weights(int64_t A, const int64_t* agreement, const int64_t* resolved,
                           double* w, void* stream);
/* Single-read iteration (what batch.reestimate runs): the consensus pass above that also
 * records the votes, then agreement from the votes alone, so P is read once per iteration.
 * vote_bits [K][A] uint64 with K = ceil(M/64): bit j of vote_bits[k][a] = (P[a][64k+j] >= 0.5);
 * cvote_words[k] bit j = market 64k+j is resolved and its consensus >= 0.5; ok_words[k] bit
 * j = market 64k+j exists and is resolved.  Counts identical to bce_reestimate_agreement. */
int bce_reestimate_consensus_votes(const double* P, int64_t A, int64_t M, int64_t ld, const double* w,
                                   double* consensus, uint8_t* null_out, uint64_t* vote_bits,
                                   uint64_t* cvote_words, uint64_t* ok_words, void* stream);
int bce_reestimate_agreement_votes(const uint64_t* vote_bits, int64_t A, int64_t M, const uint64_t* cvote_words,
                                   const uint64_t* ok_words, int64_t* agreement, int64_t* resolved,
                                   void* stream);
/* Pass 1 of the single-read iteration on the matrix cores: w^T P with
 * v_mfma_f64_16x16x4_f64 (the north star's "MFMA contraction"; batch.reestimate
 * mode="mfma" -- mode="fast" runs bce_reestimate_consensus_votes, which streams P at the same
 * HBM rate and measured faster), same outputs as
 * bce_reestimate_consensus_votes.  consensus within 4*A*2^-53 of the agent-order value;
 * markets within 8*A*2^-53 of 0.5 (or with a finite cell outside [0, 1]) are redone in agent
 * order, so vote_bits / cvote_words / ok_words -- and the agreement counts -- are identical
 * to the exact pass (a column with a NaN cell is NaN in every order and is not redone).
 * PRECONDITION of the MFMA order: every w[a] finite and >= 0.  It is checked on the device;
 * when any weight breaks it, this call computes the iteration with the exact kernel instead
 * (results identical to bce_reestimate_consensus_votes, at exact-mode speed).  scratch:
 * device buffer of bce_reestimate_mfma_scratch_bytes(M) bytes (8-byte aligned). */
int bce_reestimate_consensus_votes_mfma(const double* P, int64_t A, int64_t M, int64_t ld, const double* w,
                                        double* consensus, uint8_t* null_out, uint64_t* vote_bits,
                                        uint64_t* cvote_words, uint64_t* ok_words, void* scratch,
                                        int64_t scratch_bytes, void* stream);
int64_t bce_reestimate_mfma_scratch_bytes(int64_t M);

/* ---- JSONL front end (host C++, no GPU): SURVEY §8 f2 -----------------------------------
 *
 * Replaces, for a batch: cli._cmd_consensus_legacy / _cmd_consensus (cli.py:25-52,163-174)
 * per payload = json.load + core.validate_input_payload (core.py:24-60) + the result's
 * json.dumps(indent=2).  bce_jsonl_parse splits `text` (UTF-8; lone surrogates as 3-byte
 * sequences) on '\n', parses each non-blank line as CPython's json.loads would and runs
 * check_structure (core.py:34-58) with the reference's messages; lines it cannot restate
 * exactly get kind 2 (the caller's Python path handles them).  sourceIds of every checked
 * signal are interned over the batch in code-point order.  bce_jsonl_counts: [lines, checked
 * probabilities, names, name bytes].  bce_jsonl_arrays: per line kind (0 structure ok, 1 header
 * error, 2 hand over), first type-error index (-1), len(signals), byte span (2 x int64); the
 * CSR voff [L+1] of the checked probabilities (those before a line's first type error), their
 * values and sourceId ranks; the sorted names (bytes + [N+1] offsets).  NULL outputs skipped.
 * bce_jsonl_render: after the caller's range check (err_idx per line, bce_validate_csr) and
 * consensus launch over the computed lines (res_of: line -> row or -1; res_off: row -> CSR
 * start of its per-unique outputs; usid / nweight as bce_consensus_* writes them), every
 * line's text: "Validation error: ..." or json.dumps(result, indent=2) byte for byte (wtext:
 * per name, the JSON text of its weight object).  Call with out == NULL to render and size,
 * then with buffers to copy (text_off [L+1], ok [L]).  `threads` host threads. */
int bce_jsonl_parse(const char* text, int64_t len, int32_t threads, void** handle);
int bce_jsonl_counts(void* handle, int64_t* counts);
int bce_jsonl_arrays(void* handle, int32_t* kind, int32_t* type_err, int32_t* n_signals, int64_t* span,
                     int64_t* voff, double* prob, int32_t* sid, char* names, int64_t* name_off);
int bce_jsonl_render(void* handle, const int32_t* err_idx, const int64_t* res_of, const double* consensus,
                     const double* confidence, const double* total_weight, const int32_t* n_unique,
                     const int64_t* res_off, const int32_t* usid, const double* nweight, const char* wtext,
                     const int64_t* wtext_off, int32_t dry_run, int32_t threads, char* out, int64_t* text_off,
                     uint8_t* ok, int64_t* n_bytes);
void bce_jsonl_free(void* handle);
/* Test hook: float.__repr__ of x (the renderer's number format) into buf; returns its length. */
int32_t bce_debug_float_repr(double x, char* buf, int32_t cap);

#ifdef __cplusplus
}
#endif
#endif /* BCE_H */
