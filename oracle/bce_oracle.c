/*
 * bce_oracle.c -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY
 * (the checker for tests/, smoke() and bench.py's cpu_baseline; never the product).
 *
 * Reference: consensus-nexus/bayesian-consensus-engine, src/bayesian_engine/.
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, so a*b+c rounds twice exactly
 * like CPython).  Parity of this file with the reference is pinned by
 * tests/test_oracle_golden.py against fixtures generated from the reference itself.
 *
 * CPython semantics restated here:
 *   - builtin sum() on floats (Python <= 3.11) is a plain left-to-right double sum
 *     starting from int 0, i.e. 0.0 + x1 + x2 ...;
 *   - builtin min(a, b) returns b only if b < a; max(a, b) returns b only if b > a;
 *   - float ** float calls libm pow();  int / int true division is correctly rounded;
 *   - round(x, n) is the correctly rounded decimal (half-even on the exact binary
 *     value) converted back with strtod -- restated with glibc printf/strtod, which
 *     are exact.
 */
#include "bce_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline double py_min(double a, double b) { return (b < a) ? b : a; }
static inline double py_max(double a, double b) { return (b > a) ? b : a; }

static int cmp_u64(const void* a, const void* b) {
    uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
    return (x > y) - (x < y);
}

/* core.py:63-179 (compute_consensus) and core.py:59-60 (range check). */
int orc_consensus_csr(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                      const double* prob, const double* rel, const double* conf,
                      const uint8_t* present, int32_t n_sources, double* consensus,
                      double* confidence, double* total_weight, int32_t* n_unique,
                      int32_t* err_idx, int32_t* usid, double* weight, double* nweight) {
    int64_t cap = 0;
    uint64_t* keys = NULL;
    for (int64_t m = 0; m < n_markets; ++m) {
        const int64_t a = offsets[m], n = offsets[m + 1] - offsets[m];
        /* validate_input_payload: first signal with p < 0 or p > 1 (NaN passes). */
        int32_t e = -1;
        for (int64_t i = 0; i < n; ++i) {
            const double p = prob[a + i];
            if (p < 0 || p > 1) { e = (int32_t)i; break; }
        }
        err_idx[m] = e;
        if (n == 0) { /* core.py:88-96 no_signals */
            consensus[m] = 0.0; confidence[m] = 0.0; total_weight[m] = 0.0; n_unique[m] = 0;
            continue;
        }
        if (n > cap) {
            cap = n;
            keys = (uint64_t*)realloc(keys, (size_t)cap * sizeof(uint64_t));
            if (!keys) return -1;
        }
        for (int64_t i = 0; i < n; ++i) {
            const int32_t s = sid[a + i];
            if (s < 0 || s >= n_sources) { free(keys); return -2; }
            keys[i] = ((uint64_t)(uint32_t)s << 32) | (uint64_t)i; /* sorted(set(ids)) + input order */
        }
        qsort(keys, (size_t)n, sizeof(uint64_t), cmp_u64);
        double total = 0.0, ws = 0.0, cs = 0.0; /* core.py:107, builtin sum from 0 */
        int32_t u = 0;
        int64_t i = 0;
        while (i < n) {
            const int32_t s = (int32_t)(keys[i] >> 32);
            double psum = 0.0; /* core.py:116: sum over the source's signals in input order */
            int64_t cnt = 0;
            while (i < n && (int32_t)(keys[i] >> 32) == s) {
                psum += prob[a + (int64_t)(keys[i] & 0xffffffffu)];
                ++cnt; ++i;
            }
            const double avg = psum / (double)cnt;
            const double w = rel[s], c = conf[s]; /* core.py:110-112 (defaults baked in) */
            total += w;                            /* core.py:120 */
            ws += avg * w;                         /* core.py:135-137 */
            cs += c * w;                           /* core.py:141-143 */
            usid[a + u] = s | (present[s] ? 0 : (int32_t)0x80000000); /* core.py:167-170 */
            weight[a + u] = w;
            ++u;
        }
        n_unique[m] = u;
        total_weight[m] = total;
        if (total == 0) { /* core.py:131-133 */
            consensus[m] = 0.0;
            confidence[m] = 0.0;
        } else {
            consensus[m] = ws / total;
            confidence[m] = cs / total;
        }
        for (int32_t j = 0; j < u; ++j) /* core.py:151 */
            nweight[a + j] = (total > 0) ? weight[a + j] / total : 0.0;
    }
    free(keys);
    return 0;
}

/* libm pow, never folded or rewritten by the compiler (pow(x, 2.0) -> x*x is not what CPython
 * computes) */
static double (*volatile libm_pow)(double, double) = pow;

/* decay.py:52-58 */
double orc_decay_factor(double elapsed_days, double half_life_days) {
    if (elapsed_days <= 0) return 1.0;
    const double exponent = -elapsed_days / half_life_days;
    return libm_pow(2.0, exponent);
}

/* decay.py:90-100 */
double orc_apply_decay(double r, double elapsed_days, double half_life_days, double min_rel) {
    if (elapsed_days <= 0) return r;
    const double f = orc_decay_factor(elapsed_days, half_life_days);
    const double decayed = min_rel + (r - min_rel) * f;
    return py_max(min_rel, py_min(1.0, decayed));
}

/* decay.py:140-145: timedelta.total_seconds() == int_us / 10**6 correctly rounded. */
double orc_days_since(int64_t now_us, int64_t t_us) {
    if (t_us == ORC_NO_TIMESTAMP) return 0.0;
    const double secs = (double)(now_us - t_us) / 1e6;
    return py_max(0.0, secs / 86400.0);
}

/* reliability.py:104-140 with apply_decay=True */
void orc_decay_view(int64_t n, const double* rel, const int64_t* t_us, const uint8_t* present,
                    int64_t now_us, double half_life_days, double min_rel, double default_rel,
                    double* view) {
    for (int64_t s = 0; s < n; ++s) {
        if (!present[s]) { view[s] = default_rel; continue; }
        double r = rel[s];
        if (t_us[s] != ORC_NO_TIMESTAMP) {
            const double e = orc_days_since(now_us, t_us[s]);
            if (e > 0) r = orc_apply_decay(r, e, half_life_days, min_rel);
        }
        view[s] = r;
    }
}

/* reliability.py:161-175 */
void orc_outcome_update(int64_t n, double* rel, double* conf, int64_t* t_us, uint8_t* present,
                        const uint8_t* flags, int64_t now_us, double default_rel,
                        double default_conf) {
    for (int64_t s = 0; s < n; ++s) {
        const uint8_t f = flags[s];
        if (!(f & 1)) continue;
        const double r = present[s] ? rel[s] : default_rel;
        const double c = present[s] ? conf[s] : default_conf;
        const double direction = (f & 2) ? 1.0 : -1.0;
        const double raw = 0.15 * direction;
        const double capped = py_max(-0.10, py_min(0.10, raw));
        rel[s] = py_max(0.0, py_min(1.0, r + capped));
        conf[s] = py_min(1.0, c + (1.0 - c) * 0.10);
        t_us[s] = now_us;
        present[s] = 1;
    }
}

/* market.py:279-304 */
void orc_agreement_stats(const int64_t* offsets, int64_t n_markets, const int32_t* sid,
                         const double* prob, const int8_t* outcome, int32_t* correct,
                         int32_t* total) {
    for (int64_t m = 0; m < n_markets; ++m) {
        if (outcome[m] < 0) continue;
        for (int64_t i = offsets[m]; i < offsets[m + 1]; ++i) {
            const int predicted_true = prob[i] >= 0.5;
            total[sid[i]] += 1;
            if (predicted_true == (outcome[m] != 0)) correct[sid[i]] += 1;
        }
    }
}

/* CPython float.__round__(x, n): correctly rounded decimal, then strtod. */
double orc_round_decimal(double x, int ndigits) {
    char buf[512];
    if (!isfinite(x)) return x;
    if (fabs(x) >= 1e300) return x;
    snprintf(buf, sizeof buf, "%.*f", ndigits, x);
    return strtod(buf, NULL);
}

typedef struct {
    double key, total, confsum, maxrel;
    int32_t count;
} tb_group;

/* tiebreak.py:73-152 */
int orc_tiebreak_csr(const int64_t* offsets, int64_t n_markets, const double* pred,
                     const double* conf, const double* weight, const double* rel,
                     const double* keys, /* nullable: round(pred, 6); else the caller's round() */
                     double* winner, int32_t* label, int32_t* n_groups, double* variance,
                     double* g_key, int32_t* g_count, double* g_total, double* g_avgconf,
                     double* g_maxrel) {
    tb_group* g = NULL;
    int64_t cap = 0;
    for (int64_t m = 0; m < n_markets; ++m) {
        const int64_t a = offsets[m], n = offsets[m + 1] - offsets[m];
        if (n == 0) { /* tiebreak.py:86-87 ValueError */
            n_groups[m] = -1; winner[m] = 0.0; label[m] = -1; variance[m] = 0.0;
            continue;
        }
        if (n == 1) { /* tiebreak.py:89-96 */
            n_groups[m] = 1; winner[m] = pred[a]; label[m] = 3; variance[m] = 0.0;
            g_key[a] = pred[a]; g_count[a] = 1; g_total[a] = weight[a];
            g_avgconf[a] = conf[a]; g_maxrel[a] = rel[a];
            continue;
        }
        if (n > cap) {
            cap = n;
            g = (tb_group*)realloc(g, (size_t)cap * sizeof(tb_group));
            if (!g) return -1;
        }
        int64_t ng = 0;
        for (int64_t i = 0; i < n; ++i) { /* _group_by_prediction: dict in first-seen order */
            const double k = keys ? keys[a + i] : orc_round_decimal(pred[a + i], 6);
            int64_t j = 0;
            while (j < ng && !(g[j].key == k)) ++j;
            if (j == ng) {
                g[ng].key = k; g[ng].total = 0.0; g[ng].confsum = 0.0;
                g[ng].maxrel = rel[a + i]; g[ng].count = 0;
                ++ng;
            } else if (rel[a + i] > g[j].maxrel) {
                g[j].maxrel = rel[a + i];
            }
            g[j].total += weight[a + i];
            g[j].confsum += conf[a + i];
            g[j].count += 1;
        }
        /* confidence variance, tiebreak.py:108-110 */
        double csum = 0.0;
        for (int64_t i = 0; i < n; ++i) csum += conf[a + i];
        const double mean = csum / (double)n;
        double vs = 0.0;
        /* `(c - mean_conf) ** 2` is CPython float_pow -> libm pow, which is not correctly
         * rounded (it differs from d*d for ~0.08% of d); GCC folds pow(x, 2.0) into x*x, so
         * the call goes through a volatile pointer to stay a libm call */
        for (int64_t i = 0; i < n; ++i) vs += libm_pow(conf[a + i] - mean, 2.0);
        variance[m] = vs / (double)n;
        /* lexicographic argmax of (density, max_rel, -key); stable => first wins ties */
        int64_t best = 0;
        double bd = g[0].total / (double)g[0].count;
        for (int64_t j = 1; j < ng; ++j) {
            const double d = g[j].total / (double)g[j].count;
            int better = 0;
            if (d != bd) better = d > bd;
            else if (g[j].maxrel != g[best].maxrel) better = g[j].maxrel > g[best].maxrel;
            else better = (-g[j].key) > (-g[best].key);
            if (better) { best = j; bd = d; }
        }
        int32_t lab;
        if (ng == 1) lab = 0;
        else {
            lab = 1;
            for (int64_t j = 0; j < ng; ++j) {
                if (j == best) continue;
                const double d = g[j].total / (double)g[j].count;
                if (d == bd && g[j].maxrel == g[best].maxrel) { lab = 2; break; }
            }
        }
        winner[m] = g[best].key;
        label[m] = lab;
        n_groups[m] = (int32_t)ng;
        for (int64_t j = 0; j < ng; ++j) {
            g_key[a + j] = g[j].key;
            g_count[a + j] = g[j].count;
            g_total[a + j] = g[j].total;
            g_avgconf[a + j] = g[j].confsum / (double)g[j].count;
            g_maxrel[a + j] = g[j].maxrel;
        }
    }
    free(g);
    return 0;
}

/* composition: core.py:107-144 per market (all agents present, no duplicates) and
 * market.py:298-310 with the consensus as the pseudo-outcome. */
void orc_reestimate(const double* P, int64_t A, int64_t M, int iters, double* w,
                    double* cons_out, uint8_t* null_out, int64_t* agree_out) {
    int64_t* corr = (int64_t*)calloc((size_t)A, sizeof(int64_t));
    int64_t* tot = (int64_t*)calloc((size_t)A, sizeof(int64_t));
    for (int k = 0; k < iters; ++k) {
        double total = 0.0;
        for (int64_t ai = 0; ai < A; ++ai) total += w[ai];
        memset(corr, 0, (size_t)A * sizeof(int64_t));
        memset(tot, 0, (size_t)A * sizeof(int64_t));
        for (int64_t m = 0; m < M; ++m) {
            double ws = 0.0;
            for (int64_t ai = 0; ai < A; ++ai) ws += (0.0 + P[ai * M + m]) * w[ai];
            const int isnull = (total == 0);
            const double c = isnull ? 0.0 : ws / total;
            cons_out[(int64_t)k * M + m] = c;
            null_out[(int64_t)k * M + m] = (uint8_t)isnull;
            if (isnull) continue;
            const int outcome = c >= 0.5;
            for (int64_t ai = 0; ai < A; ++ai) {
                tot[ai] += 1;
                if ((P[ai * M + m] >= 0.5) == outcome) corr[ai] += 1;
            }
        }
        for (int64_t ai = 0; ai < A; ++ai) {
            w[ai] = tot[ai] > 0 ? (double)corr[ai] / (double)tot[ai] : 0.5;
            agree_out[(int64_t)k * A + ai] = corr[ai];
        }
    }
    free(corr);
    free(tot);
}

/* reliability_abstraction.py:119-188 (NamespacedReliabilityStore.get_reliability) for every
 * source: scopes in precedence order (market, domain, global; rel[q] == NULL = scope not
 * requested), first scope with has[q][s] wins (reliability decayed via
 * reliability.py:114-123 when apply_decay), else cold start.  scope_out 0/1/2, 3 = cold. */
void orc_namespace_resolve(int64_t n, const double* const rel[3], const double* const conf[3],
                           const int64_t* const t_us[3], const uint8_t* const has[3],
                           int apply_decay, int64_t now_us, double half_life_days, double min_rel,
                           double default_rel, double default_conf, double* rel_out,
                           double* conf_out, uint8_t* scope_out) {
    for (int64_t s = 0; s < n; ++s) {
        double r = default_rel, c = default_conf;
        int code = 3;
        for (int q = 0; q < 3; ++q) {
            if (rel[q] == NULL || !has[q][s]) continue;
            r = rel[q][s];
            c = conf[q][s];
            if (apply_decay) {
                const double e = orc_days_since(now_us, t_us[q][s]);
                if (e > 0) r = orc_apply_decay(r, e, half_life_days, min_rel);
            }
            code = q;
            break;
        }
        rel_out[s] = r;
        conf_out[s] = c;
        scope_out[s] = (uint8_t)code;
    }
}

static int cmp_f64(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return (x < y) ? -1 : (x > y) ? 1 : 0;
}

/* market.py:340-408 (CrossMarketAggregator.aggregate_consensus) per member group:
 * k = members with a consensus; sums left to right in list order from 0.0. */
void orc_aggregate_groups(const int64_t* goff, int64_t n_groups, const int64_t* members,
                          const double* cons, const double* conf, const uint8_t* has,
                          double* wavg, double* median, double* majority, double* mean_conf,
                          int64_t* n_included) {
    for (int64_t g = 0; g < n_groups; ++g) {
        double tconf = 0.0, tcons = 0.0, tprod = 0.0;
        int64_t k = 0, votes = 0;
        double* vals = (double*)malloc(sizeof(double) * (size_t)(goff[g + 1] - goff[g] + 1));
        for (int64_t i = goff[g]; i < goff[g + 1]; ++i) {
            const int64_t m = members[i];
            if (!has[m]) continue;
            tconf = tconf + conf[m];
            tcons = tcons + cons[m];
            tprod = tprod + cons[m] * conf[m];
            votes += cons[m] >= 0.5;
            vals[k++] = cons[m];
        }
        n_included[g] = k;
        if (k == 0) {
            wavg[g] = median[g] = majority[g] = mean_conf[g] = NAN;
        } else {
            wavg[g] = (tconf == 0.0) ? tcons / (double)k : tprod / tconf;
            majority[g] = (double)votes / (double)k;
            mean_conf[g] = tconf / (double)k;
            qsort(vals, (size_t)k, sizeof(double), cmp_f64);
            median[g] = vals[k / 2];
        }
        free(vals);
    }
}
