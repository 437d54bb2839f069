// jsonl.cpp -- native host half of the batched JSON front end.
//
// The reference's caller (cli.py:25-52,163-174) handles one payload per process:
// json.load -> validate_input_payload (core.py:24-60) -> compute_consensus (core.py:63-179)
// -> json.dumps(result, indent=2).  bayesian_engine.jsonl batches that over a JSONL file; in
// round 3 its Python host work (json.loads + structure checks 2.7 s, interning + assembly
// 3.3 s, rendering 2.8 s per 100k x 32 payloads) was the whole cost -- the GPU launches take
// under a millisecond.  This file moves the host work to C++ threads:
//
//   bce_jsonl_parse   split the batch into lines, parse each line as Python's json.loads
//                     would (strict RFC-8259 + NaN / Infinity / -Infinity, duplicate keys =
//                     last wins, \uXXXX with surrogate pairs combined and lone surrogates
//                     kept), run check_structure (core.py:34-58) in the reference's order
//                     with its exact messages, and collect the probabilities to range-check
//                     plus the sourceIds, interned over the whole batch in code-point order
//                     (UTF-8 byte order == Python str order, core.py:103).
//   bce_jsonl_render  after the caller's GPU launches (one range check, one consensus):
//                     each line's text -- "Validation error: ..." or the result rendered
//                     byte for byte as json.dumps(indent=2) (float repr, NaN / Infinity,
//                     encode_basestring_ascii ids, the no_signals shape, dryRun).
//
// A line this parser does not reproduce exactly is marked FALLBACK and the Python path
// handles it alone: malformed JSON (the JSONDecodeError message text is CPython's), a
// top-level value that is not an object, a non-string schemaVersion (its str() is
// CPython's), nesting deeper than 256, a blank line whose whitespace is not ASCII.  Nothing
// here is on the GPU; the arithmetic stays in the consensus kernels.
#include <locale.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bce_internal.hpp"

namespace {

enum LineKind : int32_t { kOk = 0, kHeaderError = 1, kFallback = 2 };

struct Line {
  int64_t start = 0, len = 0;   // byte span in the caller's text (without the newline)
  int32_t kind = kOk;
  int32_t type_err = -1;        // index of the first signal-level type error, -1 none
  int32_t n_checked = 0;        // probabilities before it (range-checked on the GPU)
  int32_t n_signals = 0;        // len(signals) (OK lines without a type error: == n_checked)
  std::string msg;              // header error / type error message
};

// sourceId -> local id: open addressing over 64-bit FNV-1a hashes (std::unordered_map's
// node chasing and std::hash were the parser's largest cost)
struct Intern {
  std::vector<std::string> names;
  std::vector<uint64_t> hash;   // per id
  std::vector<int32_t> slot;    // -1 empty
  size_t mask = 0;
  static uint64_t fnv(const std::string& k) {
    uint64_t h = 1469598103934665603ull;
    for (unsigned char c : k) h = (h ^ c) * 1099511628211ull;
    return h ^ (h >> 29);
  }
  void grow() {
    const size_t n = slot.empty() ? 1024 : slot.size() * 2;
    slot.assign(n, -1);
    mask = n - 1;
    for (size_t i = 0; i < names.size(); ++i) {
      size_t j = hash[i] & mask;
      while (slot[j] >= 0) j = (j + 1) & mask;
      slot[j] = (int32_t)i;
    }
  }
  int32_t id(const std::string& k) {
    if (2 * (names.size() + 1) > slot.size()) grow();
    const uint64_t h = fnv(k);
    size_t j = h & mask;
    for (;;) {
      const int32_t v = slot[j];
      if (v < 0) break;
      if (hash[(size_t)v] == h && names[(size_t)v] == k) return v;
      j = (j + 1) & mask;
    }
    const int32_t v = (int32_t)names.size();
    names.push_back(k);
    hash.push_back(h);
    slot[j] = v;
    return v;
  }
};

// One worker's share of the batch (cache-line aligned: the vectors' end pointers move on
// every push_back, and adjacent parts sharing a line serialised the workers).
struct alignas(128) Part {
  std::vector<Line> lines;
  std::vector<double> prob;      // checked probabilities of every line, in order
  std::vector<int32_t> local;    // their sourceIds as ids into `names` below
  Intern ids;
};

struct Batch {
  std::vector<Line> lines;
  std::vector<int64_t> voff;     // [L+1] CSR of the checked probabilities
  std::vector<double> prob;
  std::vector<int32_t> sid;      // rank of each checked signal's sourceId
  std::vector<std::string> names;  // sorted unique sourceIds (WTF-8)
  // rendering output
  std::string out;
  std::vector<int64_t> out_off;  // [L+1]
  std::vector<uint8_t> out_ok;   // [L]
};

// ---- JSON (CPython json.loads semantics) ------------------------------------------------
constexpr int kMaxDepth = 256;

locale_t c_locale() {
  static locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  return loc;
}

struct Parser {
  const char* p;
  const char* e;
  bool bad = false;  // anything json.loads would reject (or that we hand to Python)
  int depth = 0;

  void ws() {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
  }
  bool lit(const char* s) {
    const size_t n = strlen(s);
    if ((size_t)(e - p) >= n && memcmp(p, s, n) == 0) {
      p += n;
      return true;
    }
    return false;
  }
  static void put_cp(std::string& o, uint32_t c) {  // generalized UTF-8 (lone surrogates as 3 bytes)
    if (c < 0x80) {
      o.push_back((char)c);
    } else if (c < 0x800) {
      o.push_back((char)(0xC0 | (c >> 6)));
      o.push_back((char)(0x80 | (c & 0x3F)));
    } else if (c < 0x10000) {
      o.push_back((char)(0xE0 | (c >> 12)));
      o.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (c & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (c >> 18)));
      o.push_back((char)(0x80 | ((c >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((c >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (c & 0x3F)));
    }
  }
  int hex4(uint32_t* v) {
    if (e - p < 4) return -1;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = p[i];
      x <<= 4;
      if (c >= '0' && c <= '9') x |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') x |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') x |= (uint32_t)(c - 'A' + 10);
      else return -1;
    }
    p += 4;
    *v = x;
    return 0;
  }
  // at '"': the decoded string into *o (nullptr: validate only)
  void str(std::string* o) {
    ++p;
    if (o) o->clear();
    for (;;) {
      const char* q = p;
      while (q < e && *q != '"' && *q != '\\' && (unsigned char)*q >= 0x20) ++q;
      if (o) o->append(p, (size_t)(q - p));
      p = q;
      if (p >= e || (unsigned char)*p < 0x20) {  // unterminated / raw control character (strict)
        bad = true;
        return;
      }
      if (*p == '"') {
        ++p;
        return;
      }
      ++p;  // backslash
      if (p >= e) {
        bad = true;
        return;
      }
      const char c = *p++;
      char r = 0;
      switch (c) {
        case '"': r = '"'; break;
        case '\\': r = '\\'; break;
        case '/': r = '/'; break;
        case 'b': r = '\b'; break;
        case 'f': r = '\f'; break;
        case 'n': r = '\n'; break;
        case 'r': r = '\r'; break;
        case 't': r = '\t'; break;
        case 'u': {
          uint32_t u = 0;
          if (hex4(&u)) {
            bad = true;
            return;
          }
          // a high surrogate followed by \u low surrogate combines (json/decoder.py)
          if (u >= 0xD800 && u <= 0xDBFF && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            const char* save = p;
            p += 2;
            uint32_t lo = 0;
            if (hex4(&lo) == 0 && lo >= 0xDC00 && lo <= 0xDFFF) {
              u = 0x10000 + (((u - 0xD800) << 10) | (lo - 0xDC00));
            } else {
              p = save;  // not a pair: the next escape is decoded on its own
            }
          }
          if (o) put_cp(*o, u);
          continue;
        }
        default:
          bad = true;
          return;
      }
      if (o) o->push_back(r);
    }
  }
  // number token: value as Python would hold it (int -> float(int), with OverflowError -> inf)
  void num(double* v, bool* is_int) {
    const char* s = p;
    if (p < e && *p == '-') ++p;
    if (p < e && *p == '0') {
      ++p;
    } else if (p < e && *p >= '1' && *p <= '9') {
      while (p < e && *p >= '0' && *p <= '9') ++p;
    } else {
      bad = true;
      return;
    }
    bool integral = true;
    if (p < e && *p == '.') {
      const char* d = ++p;
      while (p < e && *p >= '0' && *p <= '9') ++p;
      if (p == d) {  // "1." is not a JSON number
        bad = true;
        return;
      }
      integral = false;
    }
    if (p < e && (*p == 'e' || *p == 'E')) {
      const char* x = p++;
      if (p < e && (*p == '+' || *p == '-')) ++p;
      const char* d = p;
      while (p < e && *p >= '0' && *p <= '9') ++p;
      if (p == d) {  // CPython's scanner then stops before the 'e': json.loads fails later
        p = x;
        bad = true;
        return;
      }
      integral = false;
    }
    *is_int = integral;
    if (!v) return;
    // Exact fast path (Clinger): a significand of <= 15 digits is an exact double and so is
    // 10^k for k <= 22, so one IEEE multiply / divide is the correctly rounded value
    {
      uint64_t sig = 0;
      int nd = 0, frac = 0, ex = 0;
      bool ok = true, seen_dot = false, nz = false;
      const char* q = (*s == '-') ? s + 1 : s;
      for (; q < p && *q != 'e' && *q != 'E'; ++q) {
        if (*q == '.') {
          seen_dot = true;
          continue;
        }
        const int d = *q - '0';
        if (d != 0 || nz) {
          nz = true;
          if (++nd > 15) {
            ok = false;
            break;
          }
        }
        sig = sig * 10 + (uint64_t)d;
        if (seen_dot) ++frac;
      }
      if (ok && q < p) {  // exponent
        ++q;
        bool eneg = false;
        if (*q == '+' || *q == '-') eneg = (*q++ == '-');
        int ev = 0;
        for (; q < p; ++q) {
          ev = ev * 10 + (*q - '0');
          if (ev > 400) {
            ok = false;
            break;
          }
        }
        ex = eneg ? -ev : ev;
      }
      const int k = ex - frac;
      if (ok && k >= -22 && k <= 22) {
        static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                       1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
        double x = (double)sig;
        x = (k >= 0) ? x * p10[k] : x / p10[-k];
        if (*s == '-' && !(integral && x == 0.0)) x = -x;  // int -0 is 0 -> float 0.0
        *v = x;
        return;
      }
    }
    // strtod in the C locale: correctly rounded like float(str) and float(int) (ties to
    // even), subnormals kept, +-inf past the double range (_as_float's OverflowError
    // branch, float('1e999')), 0 below it (float('1e-999'))
    char sb[80];
    std::string big;
    const size_t n = (size_t)(p - s);
    const char* z;
    if (n < sizeof sb) {
      memcpy(sb, s, n);
      sb[n] = 0;
      z = sb;
    } else {
      big.assign(s, n);
      z = big.c_str();
    }
    double x = strtod_l(z, nullptr, c_locale());
    if (integral && x == 0.0) x = 0.0;  // int -0 is 0 -> float 0.0
    *v = x;
  }
  // any value (validation only); returns its JSON type
  enum Type { kNull, kBool, kNum, kStr, kArr, kObj, kBad };
  Type skip() {
    ws();
    if (p >= e) {
      bad = true;
      return kBad;
    }
    const char c = *p;
    if (c == '"') {
      str(nullptr);
      return kStr;
    }
    if (c == '{' || c == '[') {
      if (++depth > kMaxDepth) {
        bad = true;
        return kBad;
      }
      const char close = (c == '{') ? '}' : ']';
      ++p;
      ws();
      if (p < e && *p == close) {
        ++p;
        --depth;
        return c == '{' ? kObj : kArr;
      }
      for (;;) {
        if (c == '{') {
          ws();
          if (p >= e || *p != '"') {
            bad = true;
            return kBad;
          }
          str(nullptr);
          if (bad) return kBad;
          ws();
          if (p >= e || *p != ':') {
            bad = true;
            return kBad;
          }
          ++p;
        }
        skip();
        if (bad) return kBad;
        ws();
        if (p < e && *p == ',') {
          ++p;
          continue;
        }
        if (p < e && *p == close) {
          ++p;
          --depth;
          return c == '{' ? kObj : kArr;
        }
        bad = true;
        return kBad;
      }
    }
    if (lit("true") || lit("false")) return kBool;
    if (lit("null")) return kNull;
    if (lit("NaN") || lit("Infinity") || lit("-Infinity")) return kNum;
    bool isi = false;
    num(nullptr, &isi);
    return bad ? kBad : kNum;
  }
};

// CPython str.isspace() code points (bidi WS/B/S or category Zs, Unicode 13 / Python 3.10)
bool py_space(uint32_t c) {
  return (c >= 0x09 && c <= 0x0D) || (c >= 0x1C && c <= 0x20) || c == 0x85 || c == 0xA0 || c == 0x1680 ||
         (c >= 0x2000 && c <= 0x200A) || c == 0x2028 || c == 0x2029 || c == 0x202F || c == 0x205F || c == 0x3000;
}

// next code point of generalized UTF-8 (our own decoded strings or the caller's text)
uint32_t next_cp(const std::string& s, size_t& i) {
  const unsigned char c = (unsigned char)s[i];
  if (c < 0x80) {
    ++i;
    return c;
  }
  int n = (c >= 0xF0) ? 3 : (c >= 0xE0) ? 2 : 1;
  uint32_t v = c & ((c >= 0xF0) ? 0x07 : (c >= 0xE0) ? 0x0F : 0x1F);
  ++i;
  for (int k = 0; k < n && i < s.size(); ++k, ++i) v = (v << 6) | ((unsigned char)s[i] & 0x3F);
  return v;
}

// s.strip() is non-empty
bool nonblank(const std::string& s) {
  for (size_t i = 0; i < s.size();)
    if (!py_space(next_cp(s, i))) return true;
  return false;
}

// One payload line (json.loads + check_structure).  Appends its checked probabilities and
// sourceId ids to the part.
void parse_line(Part& pt, const char* b, const char* e, Line& ln) {
  Parser P{b, e};
  P.ws();
  if (P.p >= P.e || *P.p != '{') {
    ln.kind = kFallback;  // not an object (or malformed): CPython's own error / TypeError
    return;
  }
  // top-level members: the last occurrence of each key wins (dict semantics)
  bool has_sv = false, sv_str = false, has_mid = false, mid_ok = false, has_sig = false;
  Parser::Type sig_type = Parser::kNull;
  const char* sig_b = nullptr;
  std::string sv, key;
  ++P.p;
  P.depth = 1;
  P.ws();
  if (P.p < P.e && *P.p == '}') {
    ++P.p;
  } else {
    for (;;) {
      P.ws();
      if (P.p >= P.e || *P.p != '"') {
        P.bad = true;
        break;
      }
      P.str(&key);
      if (P.bad) break;
      P.ws();
      if (P.p >= P.e || *P.p != ':') {
        P.bad = true;
        break;
      }
      ++P.p;
      P.ws();
      if (key == "schemaVersion") {
        has_sv = true;
        sv_str = P.p < P.e && *P.p == '"';
        if (sv_str) P.str(&sv);
        else P.skip();
      } else if (key == "marketId") {
        has_mid = true;
        if (P.p < P.e && *P.p == '"') {
          std::string mid;
          P.str(&mid);
          mid_ok = nonblank(mid);
        } else {
          P.skip();
          mid_ok = false;
        }
      } else if (key == "signals") {
        has_sig = true;
        sig_b = P.p;
        sig_type = P.skip();
      } else {
        P.skip();
      }
      if (P.bad) break;
      P.ws();
      if (P.p < P.e && *P.p == ',') {
        ++P.p;
        continue;
      }
      if (P.p < P.e && *P.p == '}') {
        ++P.p;
        break;
      }
      P.bad = true;
      break;
    }
  }
  P.ws();
  if (P.bad || P.p != P.e) {  // malformed or trailing data: json.loads' own message
    ln.kind = kFallback;
    return;
  }
  // check_structure, in the reference's order (core.py:34-46)
  if (!has_sv) {
    ln.kind = kHeaderError;
    ln.msg = "schemaVersion is required";
    return;
  }
  if (!sv_str) {
    ln.kind = kFallback;  // the message would hold str(value): CPython formats it
    return;
  }
  if (sv != "1.0.0") {
    ln.kind = kHeaderError;
    ln.msg = "schemaVersion must be '1.0.0' (got '" + sv + "')";
    return;
  }
  if (!has_mid) {
    ln.kind = kHeaderError;
    ln.msg = "marketId is required";
    return;
  }
  if (!mid_ok) {
    ln.kind = kHeaderError;
    ln.msg = "marketId must be a non-empty string";
    return;
  }
  if (!has_sig) {
    ln.kind = kHeaderError;
    ln.msg = "signals is required";
    return;
  }
  if (sig_type != Parser::kArr) {
    ln.kind = kHeaderError;
    ln.msg = "signals must be an array";
    return;
  }
  // the signals array, again from its start (already validated): per signal, the last
  // sourceId / probability member wins; the first type error stops the loop (core.py:48-58)
  Parser S{sig_b, e};
  ++S.p;  // '['
  S.ws();
  int idx = 0;
  std::string sidv;
  bool stopped = false;
  if (S.p < S.e && *S.p == ']') {
    ln.n_signals = 0;
  } else {
    for (;; ++idx) {
      S.ws();
      if (!stopped) {
        if (*S.p != '{') {
          ln.type_err = idx;
          ln.msg = "signals[" + std::to_string(idx) + "] must be an object";
          stopped = true;
          S.skip();
        } else {
          bool has_s = false, s_str = false, has_p = false, p_num = false;
          double pv = 0.0;
          ++S.p;
          S.ws();
          if (*S.p == '}') {
            ++S.p;
          } else {
            for (;;) {
              S.ws();
              S.str(&key);
              S.ws();
              ++S.p;  // ':'
              S.ws();
              if (key == "sourceId") {
                has_s = true;
                s_str = *S.p == '"';
                if (s_str) S.str(&sidv);
                else S.skip();
              } else if (key == "probability") {
                has_p = true;
                const char c = *S.p;
                p_num = true;
                if (c == 't' || c == 'f') {
                  pv = (c == 't') ? 1.0 : 0.0;  // bool is an int (core.py:57)
                  S.skip();
                } else if (S.lit("NaN")) {
                  pv = NAN;
                } else if (S.lit("Infinity")) {
                  pv = HUGE_VAL;
                } else if (S.lit("-Infinity")) {
                  pv = -HUGE_VAL;
                } else if (c == '-' || (c >= '0' && c <= '9')) {
                  bool isi = false;
                  S.num(&pv, &isi);
                } else {
                  p_num = false;
                  S.skip();
                }
              } else {
                S.skip();
              }
              S.ws();
              if (*S.p == ',') {
                ++S.p;
                continue;
              }
              ++S.p;  // '}'
              break;
            }
          }
          const char* why = nullptr;
          if (!has_s) why = "sourceId is required";
          else if (!s_str || !nonblank(sidv)) why = ".sourceId must be a non-empty string";
          else if (!has_p) why = "probability is required";
          else if (!p_num) why = ".probability must be a number";
          if (why) {
            ln.type_err = idx;
            ln.msg = (why[0] == '.') ? "signals[" + std::to_string(idx) + "]" + why : std::string(why);
            stopped = true;
          } else {
            const int32_t id = pt.ids.id(sidv);
            pt.prob.push_back(pv);
            pt.local.push_back(id);
            ++ln.n_checked;
          }
        }
      } else {
        S.skip();
      }
      S.ws();
      if (*S.p == ',') {
        ++S.p;
        continue;
      }
      break;  // ']'
    }
    ln.n_signals = idx + 1;
  }
}

// ---- rendering (json.dumps(indent=2) of the computed result; jsonl.render's layout) -------
void put_u64(std::string& o, uint64_t v) {
  char b[24];
  auto r = std::to_chars(b, b + sizeof b, v);
  o.append(b, r.ptr);
}

// float.__repr__ (PyOS_double_to_string(x, 'r', 0, Py_DTSF_ADD_DOT_0)): shortest round-trip
// digits; exponent form when the decimal point falls before -4 or after 16 digits
void put_repr(std::string& o, double x) {
  if (x != x) {
    o += "NaN";
    return;
  }
  if (x == HUGE_VAL) {
    o += "Infinity";
    return;
  }
  if (x == -HUGE_VAL) {
    o += "-Infinity";
    return;
  }
  char b[64];
  auto r = std::to_chars(b, b + sizeof b, x, std::chars_format::scientific);
  std::string_view s(b, (size_t)(r.ptr - b));
  bool neg = false;
  if (!s.empty() && s[0] == '-') {
    neg = true;
    s.remove_prefix(1);
  }
  const size_t epos = s.find('e');
  std::string digits;
  digits.push_back(s[0]);
  if (epos > 1) digits.append(s.substr(2, epos - 2));  // skip "d."
  int ex = 0;
  std::from_chars(s.data() + epos + 1 + (s[epos + 1] == '+'), s.data() + s.size(), ex);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  const int nd = (int)digits.size();
  const int decpt = ex + 1;
  if (neg) o.push_back('-');
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      o += "0.";
      o.append((size_t)(-decpt), '0');
      o += digits;
    } else if (decpt >= nd) {
      o += digits;
      o.append((size_t)(decpt - nd), '0');
      o += ".0";
    } else {
      o.append(digits, 0, (size_t)decpt);
      o.push_back('.');
      o.append(digits, (size_t)decpt, std::string::npos);
    }
  } else {
    o.push_back(digits[0]);
    if (nd > 1) {
      o.push_back('.');
      o.append(digits, 1, std::string::npos);
    }
    o.push_back('e');
    const int e2 = decpt - 1;
    o.push_back(e2 < 0 ? '-' : '+');
    const int ae = e2 < 0 ? -e2 : e2;
    if (ae < 10) o.push_back('0');
    put_u64(o, (uint64_t)ae);
  }
}

// json.encoder.encode_basestring_ascii of a (generalized UTF-8) string
void put_qstr(std::string& o, const std::string& s) {
  static const char* hx = "0123456789abcdef";
  auto u4 = [&](uint32_t c) {
    o += "\\u";
    o.push_back(hx[(c >> 12) & 15]);
    o.push_back(hx[(c >> 8) & 15]);
    o.push_back(hx[(c >> 4) & 15]);
    o.push_back(hx[c & 15]);
  };
  o.push_back('"');
  for (size_t i = 0; i < s.size();) {
    const uint32_t c = next_cp(s, i);
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      default:
        if (c >= 0x20 && c < 0x7F) {
          o.push_back((char)c);
        } else if (c < 0x10000) {
          u4(c);
        } else {
          const uint32_t v = c - 0x10000;
          u4(0xD800 | (v >> 10));
          u4(0xDC00 | (v & 0x3FF));
        }
    }
  }
  o.push_back('"');
}

struct RenderIn {
  const int32_t* err_idx;  // [L] GPU range check: first bad index among the checked probs, -1
  const int64_t* res_of;   // [L] row in the consensus outputs for lines that were computed, -1
  const double* consensus;
  const double* confidence;
  const double* total_weight;
  const int32_t* n_unique;
  const int64_t* res_off;  // [R+1] per computed row: start of its per-unique outputs
  const int32_t* usid;
  const double* nweight;
  const char* wtext;       // weight texts (json of each name's reliability object)
  const int64_t* wtext_off;
  int32_t dry_run;
};

void render_line(std::string& o, const Batch& B, const Line& ln, int64_t l, const RenderIn& in, bool* ok) {
  *ok = false;
  if (ln.kind == kHeaderError) {
    o += "Validation error: ";
    o += ln.msg;
    return;
  }
  const int32_t ek = in.err_idx[l];
  if (ek >= 0) {  // a range error before the first type error wins (core.py:59-60)
    o += "Validation error: signals[";
    put_u64(o, (uint64_t)ek);
    o += "].probability must be between 0 and 1";
    return;
  }
  if (ln.type_err >= 0) {
    o += "Validation error: ";
    o += ln.msg;
    return;
  }
  *ok = true;
  const char* dry = in.dry_run ? ",\n    \"dryRun\": true" : "";
  if (ln.n_signals == 0) {  // core.py:88-96
    o += "{\n  \"schemaVersion\": \"1.0.0\",\n  \"consensus\": null,\n  \"confidence\": 0.0,\n  \"sourceWeights\": [],\n"
         "  \"normalization\": {\n    \"totalWeight\": 0.0,\n    \"sourceCount\": 0\n  },\n"
         "  \"diagnostics\": {\n    \"status\": \"no_signals\",\n    \"sources\": 0";
    o += dry;
    o += "\n  }\n}";
    return;
  }
  const int64_t r = in.res_of[l];
  const double tw = in.total_weight[r];
  const bool null_ = tw == 0.0;  // core.py:131
  const int32_t u = in.n_unique[r];
  const int64_t base = in.res_off[r];
  o += "{\n  \"schemaVersion\": \"1.0.0\",\n  \"consensus\": ";
  if (null_) o += "null";
  else put_repr(o, in.consensus[r]);
  o += ",\n  \"confidence\": ";
  if (null_) o += "0.0";
  else put_repr(o, in.confidence[r]);
  o += ",\n  \"sourceWeights\": ";
  if (u == 0) {
    o += "[]";
  } else {
    o += "[\n";
    for (int32_t j = 0; j < u; ++j) {
      const int32_t k = in.usid[base + j] & 0x7FFFFFFF;
      o += "    {\n      \"sourceId\": ";
      put_qstr(o, B.names[(size_t)k]);
      o += ",\n      \"weight\": ";
      o.append(in.wtext + in.wtext_off[k], (size_t)(in.wtext_off[k + 1] - in.wtext_off[k]));
      o += ",\n      \"normalizedWeight\": ";
      put_repr(o, in.nweight[base + j]);
      o += (j + 1 < u) ? "\n    },\n" : "\n    }\n  ]";
    }
  }
  o += ",\n  \"normalization\": {\n    \"totalWeight\": ";
  put_repr(o, tw);
  o += ",\n    \"sourceCount\": ";
  put_u64(o, (uint64_t)u);
  o += "\n  },\n  \"diagnostics\": {\n    \"status\": \"computed\",\n    \"sources\": ";
  put_u64(o, (uint64_t)ln.n_signals);
  o += ",\n    \"uniqueSources\": ";
  put_u64(o, (uint64_t)u);
  o += ",\n    \"coldStartSources\": ";
  bool any = false;
  for (int32_t j = 0; j < u; ++j) {
    const int32_t v = in.usid[base + j];
    if (v >= 0) continue;
    o += any ? ",\n      " : "[\n      ";
    any = true;
    put_qstr(o, B.names[(size_t)(v & 0x7FFFFFFF)]);
  }
  o += any ? "\n    ]" : "[]";
  o += dry;
  o += "\n  }\n}";
}

template <class F>
void parallel(int64_t n, int threads, F&& f) {
  if (threads <= 1 || n < 2048) {
    f(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int w = 0; w < threads; ++w) {
    const int64_t a = n * w / threads, b = n * (w + 1) / threads;
    th.emplace_back([&f, w, a, b] { f(w, a, b); });
  }
  for (auto& t : th) t.join();
}

}  // namespace

using namespace bce;

extern "C" int bce_jsonl_parse(const char* text, int64_t len, int32_t threads, void** handle) {
  BCE_REQUIRE(handle && (text || len == 0) && len >= 0, "jsonl_parse: bad argument");
  auto* B = new Batch();
  // line spans (a blank line -- only ASCII whitespace -- is skipped, as `line.strip()` does;
  // other whitespace-only lines go to the Python path)
  std::vector<std::pair<int64_t, int64_t>> spans;
  for (int64_t i = 0; i < len;) {
    const char* nl = (const char*)memchr(text + i, '\n', (size_t)(len - i));
    const int64_t j = nl ? (int64_t)(nl - text) : len;
    int64_t k = i;
    while (k < j && (text[k] == ' ' || text[k] == '\t' || text[k] == '\r' || text[k] == '\v' || text[k] == '\f')) ++k;
    if (k < j) spans.emplace_back(i, j - i);
    i = j + 1;
  }
  const int64_t L = (int64_t)spans.size();
  const int T = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  const int nparts = (L >= 2048) ? T : 1;
  std::vector<Part> parts((size_t)nparts);
  parallel(L, nparts, [&](int w, int64_t a, int64_t b) {
    Part& pt = parts[(size_t)w];
    pt.lines.resize((size_t)(b - a));
    for (int64_t l = a; l < b; ++l) {
      Line& ln = pt.lines[(size_t)(l - a)];
      ln.start = spans[(size_t)l].first;
      ln.len = spans[(size_t)l].second;
      const char* s = text + ln.start;
      const char* e = s + ln.len;
      bool ascii_blank = true;
      for (const char* q = s; q < e; ++q)
        if (!(*q == ' ' || *q == '\t' || *q == '\r' || *q == '\v' || *q == '\f')) ascii_blank = false;
      if (ascii_blank) continue;  // unreachable (filtered above)
      const size_t np = pt.prob.size();
      parse_line(pt, s, e, ln);
      if (ln.kind != kOk) {  // nothing of a header-error / fallback line is range-checked
        pt.prob.resize(np);
        pt.local.resize(np);
        ln.n_checked = 0;
      }
    }
  });
  // merge: lines in order, every name interned once, ranks in byte (== code point) order
  std::unordered_map<std::string_view, int32_t> all;
  std::vector<std::string_view> uniq;
  for (auto& pt : parts)
    for (auto& nm : pt.ids.names)
      if (all.emplace(std::string_view(nm), 0).second) uniq.push_back(std::string_view(nm));
  std::sort(uniq.begin(), uniq.end());
  B->names.reserve(uniq.size());
  for (size_t i = 0; i < uniq.size(); ++i) {
    all[uniq[i]] = (int32_t)i;
    B->names.emplace_back(uniq[i]);
  }
  B->lines.reserve((size_t)L);
  B->voff.assign((size_t)L + 1, 0);
  int64_t nv = 0;
  for (auto& pt : parts) {
    for (auto& ln : pt.lines) {
      B->lines.push_back(std::move(ln));
      nv += B->lines.back().n_checked;
      B->voff[B->lines.size()] = nv;
    }
  }
  B->prob.resize((size_t)nv);
  B->sid.resize((size_t)nv);
  int64_t at = 0;
  for (auto& pt : parts) {
    std::vector<int32_t> rank(pt.ids.names.size());
    for (size_t i = 0; i < pt.ids.names.size(); ++i) rank[i] = all[std::string_view(pt.ids.names[i])];
    for (size_t i = 0; i < pt.prob.size(); ++i) {
      B->prob[(size_t)at] = pt.prob[i];
      B->sid[(size_t)at] = rank[(size_t)pt.local[i]];
      ++at;
    }
  }
  *handle = B;
  return BCE_OK;
}

// counts: [0] lines, [1] checked probabilities, [2] names, [3] bytes of all names
extern "C" int bce_jsonl_counts(void* handle, int64_t* counts) {
  BCE_REQUIRE(handle && counts, "jsonl_counts: NULL");
  const Batch* B = (const Batch*)handle;
  counts[0] = (int64_t)B->lines.size();
  counts[1] = (int64_t)B->prob.size();
  counts[2] = (int64_t)B->names.size();
  int64_t nb = 0;
  for (auto& s : B->names) nb += (int64_t)s.size();
  counts[3] = nb;
  return BCE_OK;
}

// per line: kind (0 structure ok, 1 header error, 2 Python fallback), first type-error index
// (-1), len(signals), byte span; the CSR of checked probabilities with their sourceId ranks;
// the sorted names (concatenated, with [N+1] offsets).  Any output pointer may be NULL.
extern "C" int bce_jsonl_arrays(void* handle, int32_t* kind, int32_t* type_err, int32_t* n_signals,
                                int64_t* span, int64_t* voff, double* prob, int32_t* sid, char* names,
                                int64_t* name_off) {
  BCE_REQUIRE(handle, "jsonl_arrays: NULL handle");
  const Batch* B = (const Batch*)handle;
  const size_t L = B->lines.size();
  for (size_t l = 0; l < L; ++l) {
    const Line& ln = B->lines[l];
    if (kind) kind[l] = ln.kind;
    if (type_err) type_err[l] = ln.type_err;
    if (n_signals) n_signals[l] = ln.n_signals;
    if (span) {
      span[2 * l] = ln.start;
      span[2 * l + 1] = ln.len;
    }
  }
  if (voff) memcpy(voff, B->voff.data(), (L + 1) * sizeof(int64_t));
  if (prob && !B->prob.empty()) memcpy(prob, B->prob.data(), B->prob.size() * sizeof(double));
  if (sid && !B->sid.empty()) memcpy(sid, B->sid.data(), B->sid.size() * sizeof(int32_t));
  if (names && name_off) {
    int64_t at = 0;
    name_off[0] = 0;
    for (size_t i = 0; i < B->names.size(); ++i) {
      memcpy(names + at, B->names[i].data(), B->names[i].size());
      at += (int64_t)B->names[i].size();
      name_off[i + 1] = at;
    }
  }
  return BCE_OK;
}

// Every line's text (without newline) into one buffer; out_len / n_bytes report its size.
// Call with out == NULL to render and get the size, then again with a buffer to copy.
extern "C" int bce_jsonl_render(void* handle, const int32_t* err_idx, const int64_t* res_of,
                                const double* consensus, const double* confidence, const double* total_weight,
                                const int32_t* n_unique, const int64_t* res_off, const int32_t* usid,
                                const double* nweight, const char* wtext, const int64_t* wtext_off,
                                int32_t dry_run, int32_t threads, char* out, int64_t* text_off, uint8_t* ok,
                                int64_t* n_bytes) {
  BCE_REQUIRE(handle && n_bytes, "jsonl_render: NULL");
  Batch* B = (Batch*)handle;
  const int64_t L = (int64_t)B->lines.size();
  if (!out) {
    BCE_REQUIRE(L == 0 || (err_idx && res_of), "jsonl_render: NULL inputs");
    const RenderIn in{err_idx, res_of, consensus, confidence, total_weight, n_unique, res_off, usid, nweight,
                      wtext, wtext_off, dry_run};
    const int T = (L >= 2048) ? (threads < 1 ? 1 : (threads > 64 ? 64 : threads)) : 1;
    std::vector<std::string> bufs((size_t)T);
    std::vector<int64_t> loc((size_t)L + 1, 0);
    B->out_ok.assign((size_t)L, 0);
    parallel(L, T, [&](int w, int64_t a, int64_t b) {
      std::string& o = bufs[(size_t)w];
      for (int64_t l = a; l < b; ++l) {
        bool good = false;
        if (B->lines[(size_t)l].kind != kFallback) render_line(o, *B, B->lines[(size_t)l], l, in, &good);
        B->out_ok[(size_t)l] = good ? 1 : 0;
        loc[(size_t)l + 1] = (int64_t)o.size();  // end within this worker's buffer
      }
    });
    B->out.clear();
    B->out_off.assign((size_t)L + 1, 0);
    size_t total = 0;
    for (auto& s : bufs) total += s.size();
    B->out.reserve(total);
    int64_t l = 0;
    for (int w = 0; w < T; ++w) {
      const int64_t a = (T == 1) ? 0 : L * w / T, b = (T == 1) ? L : L * (w + 1) / T;
      const int64_t shift = (int64_t)B->out.size();
      int64_t prev = 0;
      for (l = a; l < b; ++l) {
        B->out_off[(size_t)l] = shift + prev;
        prev = loc[(size_t)l + 1];
      }
      B->out += bufs[(size_t)w];
    }
    B->out_off[(size_t)L] = (int64_t)B->out.size();
    *n_bytes = (int64_t)B->out.size();
    return BCE_OK;
  }
  memcpy(out, B->out.data(), B->out.size());
  if (text_off) memcpy(text_off, B->out_off.data(), (size_t)(L + 1) * sizeof(int64_t));
  if (ok && L > 0) memcpy(ok, B->out_ok.data(), (size_t)L);  // L == 0: data() may be NULL (UBSan)
  *n_bytes = (int64_t)B->out.size();
  return BCE_OK;
}

extern "C" void bce_jsonl_free(void* handle) { delete (Batch*)handle; }

// float.__repr__ of x into buf (test hook for the renderer's number format); returns length
extern "C" int32_t bce_debug_float_repr(double x, char* buf, int32_t cap) {
  std::string o;
  put_repr(o, x);
  const int32_t n = (int32_t)o.size();
  if (buf && cap > n) {
    memcpy(buf, o.data(), (size_t)n);
    buf[n] = 0;
  }
  return n;
}
