// dkm_io.cpp -- host-side text parsers behind dislib's Dataset loaders
// (SURVEY.md section 8, row f1).  Plain C++ (no device code): the loaders
// sit before the k-means path, and their output (CSR / dense fp64) is
// uploaded once into HBM by the Python layer.
//
// Reference behaviour being replaced:
//  * dislib/data/base.py:224-238 `_read_libsvm` -> sklearn 1.7.2
//    `load_svmlight_file` (sklearn/datasets/_svmlight_format_fast.pyx
//    `_load_svmlight_file`): '#' starts a comment, tokens split on ASCII
//    whitespace, blank lines skipped, target = float(tok0), an optional
//    leading "qid:" feature is skipped, each feature is "idx:value" with
//    idx = int(...), value = float(...); idx < 0 and idx <= previous idx
//    are errors.  The zero/one-based "auto" shift and the n_features check
//    are per-chunk numpy steps done by the caller.
//  * dislib/data/base.py:188 / :212 `np.genfromtxt(lines, delimiter)`:
//    comment cut at '#', strip " \r\n", skip empty lines, split at the
//    delimiter (or whitespace runs), float() of each field, anything that
//    does not convert (or an empty field) is NaN, a row with a different
//    number of fields than the first row is an error.
//  * dislib/data/base.py:150-158: files are read in text mode, so "\n",
//    "\r\n" and a lone "\r" all end a line; chunks count raw lines
//    (blank and comment lines included), hence `row_line` below.
//
// Both formats are parsed in two passes over T byte ranges cut at line
// starts (count, prefix-sum, fill), one std::thread per range.  Numbers are
// converted with strtod/strtoll (correctly rounded, like Python's float and
// int), after rejecting the spellings Python refuses (hex, "nan(...)").
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dkm.h"

namespace dkm {
int fail(int code, const std::string &msg);
}

namespace {

inline bool is_ws(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' ||
         c == '\f';
}
inline bool is_eol(char c) { return c == '\n' || c == '\r'; }

// First line start at or after byte p (universal newlines).
int64_t line_start_at(const char *b, int64_t len, int64_t p) {
  if (p <= 0) return 0;
  for (int64_t q = p; q < len; ++q) {
    char prev = b[q - 1];
    if (prev == '\n' || (prev == '\r' && b[q] != '\n')) return q;
  }
  return len;
}

// End of the line starting at s, and the start of the next one.
inline int64_t line_end(const char *b, int64_t len, int64_t s, int64_t *next) {
  int64_t e = s;
  while (e < len && !is_eol(b[e])) ++e;
  int64_t nx = e;
  if (nx < len) nx += (b[nx] == '\r' && nx + 1 < len && b[nx + 1] == '\n') ? 2 : 1;
  *next = nx;
  return e;
}

std::vector<int64_t> split_ranges(const char *b, int64_t len, int nthreads) {
  int T = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  T = std::max(1, std::min(T, 64));
  if (len < ((int64_t)1 << 20)) T = 1;  // small inputs: one range
  std::vector<int64_t> cut(T + 1);
  for (int t = 0; t <= T; ++t)
    cut[t] = t == T ? len : line_start_at(b, len, len * t / T);
  return cut;
}

template <class F>
void run_threads(int T, F f) {
  if (T == 1) {
    f(0);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t) th.emplace_back(f, t);
  for (auto &x : th) x.join();
}

// Python float() on the bytes [p, p+n): surrounding whitespace allowed,
// no hex, no "nan(...)".  Returns false if Python would raise.
bool py_float(const char *p, int64_t n, double *out) {
  while (n > 0 && is_ws(*p)) ++p, --n;
  while (n > 0 && is_ws(p[n - 1])) --n;
  if (n <= 0) return false;
  char small[96];
  std::string big;
  const char *s;
  if (n < (int64_t)sizeof(small)) {
    memcpy(small, p, n);
    small[n] = 0;
    s = small;
  } else {
    big.assign(p, n);
    s = big.c_str();
  }
  for (int64_t i = 0; i < n; ++i)
    if (s[i] == 'x' || s[i] == 'X' || s[i] == '(' || s[i] == 'p' ||
        s[i] == 'P')
      return false;
  char *end = nullptr;
  double v = strtod(s, &end);
  if (end != s + n) return false;
  *out = v;
  return true;
}

// Python int() on [p, p+n) into an int32 (the Cython parser's `cdef int`).
bool py_int32(const char *p, int64_t n, int64_t *out) {
  while (n > 0 && is_ws(*p)) ++p, --n;
  while (n > 0 && is_ws(p[n - 1])) --n;
  if (n <= 0 || n > 40) return false;
  char s[48];
  memcpy(s, p, n);
  s[n] = 0;
  char *end = nullptr;
  long long v = strtoll(s, &end, 10);
  if (end != s + n) return false;
  if (v > INT32_MAX || v < INT32_MIN) return false;
  *out = v;
  return true;
}

struct Tok {
  int64_t b, e;
};

// Tokens of a libsvm line [s, e) after the comment cut.
inline int tokenize_ws(const char *b, int64_t s, int64_t e,
                       std::vector<Tok> *toks) {
  toks->clear();
  int64_t i = s;
  while (i < e) {
    while (i < e && is_ws(b[i])) ++i;
    if (i >= e) break;
    int64_t j = i;
    while (j < e && !is_ws(b[j])) ++j;
    toks->push_back({i, j});
    i = j;
  }
  return (int)toks->size();
}

inline int64_t comment_cut(const char *b, int64_t s, int64_t e) {
  const void *h = memchr(b + s, '#', (size_t)(e - s));
  return h ? (const char *)h - b : e;
}

inline bool is_qid(const char *b, const Tok &t) {
  return t.e - t.b >= 3 && b[t.b] == 'q' && b[t.b + 1] == 'i' &&
         b[t.b + 2] == 'd';
}

struct Err {
  int64_t line = -1;
  std::string msg;
};

int report(const std::vector<Err> &errs) {
  const Err *first = nullptr;
  for (auto &e : errs)
    if (e.line >= 0 && (!first || e.line < first->line)) first = &e;
  if (!first) return 0;
  return dkm::fail(DKM_E_PARSE,
                   first->msg + " (line " + std::to_string(first->line + 1) +
                       ")");
}

}  // namespace

extern "C" {

int dkm_libsvm_count(const char *buf, int64_t len, int nthreads,
                     int64_t *counts) {
  if (!counts || len < 0 || (len > 0 && !buf))
    return dkm::fail(DKM_E_ARG, "libsvm_count: bad arguments");
  auto cut = split_ranges(buf, len, nthreads);
  int T = (int)cut.size() - 1;
  std::vector<int64_t> c(3 * T, 0);
  run_threads(T, [&](int t) {
    std::vector<Tok> toks;
    int64_t lines = 0, rows = 0, nnz = 0, nx;
    for (int64_t s = cut[t]; s < cut[t + 1]; s = nx) {
      int64_t e = line_end(buf, len, s, &nx);
      ++lines;
      int n = tokenize_ws(buf, s, comment_cut(buf, s, e), &toks);
      if (n == 0) continue;
      ++rows;
      nnz += n - 1 - ((n > 1 && is_qid(buf, toks[1])) ? 1 : 0);
    }
    c[3 * t] = lines, c[3 * t + 1] = rows, c[3 * t + 2] = nnz;
  });
  counts[0] = counts[1] = counts[2] = 0;
  for (int t = 0; t < T; ++t)
    for (int j = 0; j < 3; ++j) counts[j] += c[3 * t + j];
  counts[3] = T;
  return 0;
}

int dkm_libsvm_parse(const char *buf, int64_t len, int nthreads,
                     int64_t *indptr, int32_t *indices, double *data,
                     double *y, int64_t *row_line) {
  if (len < 0 || (len > 0 && !buf) || !indptr)
    return dkm::fail(DKM_E_ARG, "libsvm_parse: bad arguments");
  auto cut = split_ranges(buf, len, nthreads);
  int T = (int)cut.size() - 1;
  // pass 1: per-range counts (same tokenizer as dkm_libsvm_count)
  std::vector<int64_t> L(T + 1, 0), R(T + 1, 0), Z(T + 1, 0);
  run_threads(T, [&](int t) {
    std::vector<Tok> toks;
    int64_t lines = 0, rows = 0, nnz = 0, nx;
    for (int64_t s = cut[t]; s < cut[t + 1]; s = nx) {
      int64_t e = line_end(buf, len, s, &nx);
      ++lines;
      int n = tokenize_ws(buf, s, comment_cut(buf, s, e), &toks);
      if (n == 0) continue;
      ++rows;
      nnz += n - 1 - ((n > 1 && is_qid(buf, toks[1])) ? 1 : 0);
    }
    L[t + 1] = lines, R[t + 1] = rows, Z[t + 1] = nnz;
  });
  for (int t = 0; t < T; ++t)
    L[t + 1] += L[t], R[t + 1] += R[t], Z[t + 1] += Z[t];
  if ((R[T] > 0 && (!y || !row_line)) || (Z[T] > 0 && (!indices || !data)))
    return dkm::fail(DKM_E_ARG, "libsvm_parse: NULL output");
  // pass 2: fill
  std::vector<Err> errs(T);
  run_threads(T, [&](int t) {
    std::vector<Tok> toks;
    int64_t line = L[t], row = R[t], z = Z[t], nx;
    Err &err = errs[t];
    for (int64_t s = cut[t]; s < cut[t + 1]; s = nx, ++line) {
      int64_t e = line_end(buf, len, s, &nx);
      int n = tokenize_ws(buf, s, comment_cut(buf, s, e), &toks);
      if (n == 0) continue;
      double tv;
      if (!py_float(buf + toks[0].b, toks[0].e - toks[0].b, &tv)) {
        err.line = line;
        err.msg = "could not convert string to float: '" +
                  std::string(buf + toks[0].b, toks[0].e - toks[0].b) + "'";
        return;
      }
      y[row] = tv;
      row_line[row] = line;
      int f0 = (n > 1 && is_qid(buf, toks[1])) ? 2 : 1;
      int64_t prev = -1;
      for (int i = f0; i < n; ++i) {
        const Tok &k = toks[i];
        const char *colon =
            (const char *)memchr(buf + k.b, ':', (size_t)(k.e - k.b));
        if (!colon) {
          err.line = line;
          err.msg = "not enough values to unpack (expected 2, got 1)";
          return;
        }
        int64_t ci = colon - buf, idx;
        if (!py_int32(buf + k.b, ci - k.b, &idx)) {
          err.line = line;
          err.msg = "invalid literal for int() with base 10: '" +
                    std::string(buf + k.b, ci - k.b) + "'";
          return;
        }
        if (idx < 0) {
          err.line = line;
          err.msg = "Invalid index " + std::to_string(idx) +
                    " in SVMlight/LibSVM data file.";
          return;
        }
        if (idx <= prev) {
          err.line = line;
          err.msg = "Feature indices in SVMlight/LibSVM data file should be "
                    "sorted and unique.";
          return;
        }
        double v;
        if (!py_float(buf + ci + 1, k.e - ci - 1, &v)) {
          err.line = line;
          err.msg = "could not convert string to float: '" +
                    std::string(buf + ci + 1, k.e - ci - 1) + "'";
          return;
        }
        indices[z] = (int32_t)idx;
        data[z] = v;
        ++z;
        prev = idx;
      }
      ++row;
      indptr[row] = z;
    }
  });
  indptr[0] = 0;
  return report(errs);
}

// genfromtxt's field split of one line: returns the number of fields and
// (if out != NULL) converts them.  delim == 0: whitespace runs.
static int64_t txt_fields(const char *b, int64_t s, int64_t e, char delim,
                          double *out, int64_t cap) {
  e = comment_cut(b, s, e);
  while (s < e && (b[s] == ' ' || b[s] == '\r' || b[s] == '\n')) ++s;
  while (e > s && (b[e - 1] == ' ' || b[e - 1] == '\r' || b[e - 1] == '\n'))
    --e;
  if (s >= e) return 0;
  int64_t nf = 0;
  if (delim == 0) {
    int64_t i = s;
    while (i < e) {
      while (i < e && is_ws(b[i])) ++i;
      if (i >= e) break;
      int64_t j = i;
      while (j < e && !is_ws(b[j])) ++j;
      if (out && nf < cap) {
        double v;
        out[nf] = py_float(b + i, j - i, &v) ? v : __builtin_nan("");
      }
      ++nf;
      i = j;
    }
    return nf;
  }
  int64_t i = s;
  for (;;) {
    const void *h = memchr(b + i, delim, (size_t)(e - i));
    int64_t j = h ? (const char *)h - b : e;
    if (out && nf < cap) {
      double v;
      out[nf] = py_float(b + i, j - i, &v) ? v : __builtin_nan("");
    }
    ++nf;
    if (!h) break;
    i = j + 1;
  }
  return nf;
}

int dkm_txt_count(const char *buf, int64_t len, int delimiter, int nthreads,
                  int64_t *counts) {
  if (!counts || len < 0 || (len > 0 && !buf) || delimiter < 0 ||
      delimiter > 255)
    return dkm::fail(DKM_E_ARG, "txt_count: bad arguments");
  char dl = (char)delimiter;
  auto cut = split_ranges(buf, len, nthreads);
  int T = (int)cut.size() - 1;
  // per range: lines, rows, first row's field count (+ its line)
  std::vector<int64_t> c(4 * T, 0);
  run_threads(T, [&](int t) {
    int64_t lines = 0, rows = 0, ncol = -1, ncol_line = -1, nx;
    for (int64_t s = cut[t]; s < cut[t + 1]; s = nx) {
      int64_t e = line_end(buf, len, s, &nx);
      int64_t nf = txt_fields(buf, s, e, dl, nullptr, 0);
      if (nf > 0) {
        if (ncol < 0) ncol = nf, ncol_line = lines;
        ++rows;
      }
      ++lines;
    }
    c[4 * t] = lines, c[4 * t + 1] = rows, c[4 * t + 2] = ncol,
           c[4 * t + 3] = ncol_line;
  });
  counts[0] = counts[1] = 0;
  counts[2] = 0;
  bool have = false;
  for (int t = 0; t < T; ++t) {
    if (!have && c[4 * t + 2] >= 0) counts[2] = c[4 * t + 2], have = true;
    counts[0] += c[4 * t], counts[1] += c[4 * t + 1];
  }
  counts[3] = T;
  return 0;
}

int dkm_txt_parse(const char *buf, int64_t len, int delimiter, int64_t n_cols,
                  int nthreads, double *out, int64_t *row_line) {
  if (len < 0 || (len > 0 && !buf) || n_cols < 0 || delimiter < 0 ||
      delimiter > 255)
    return dkm::fail(DKM_E_ARG, "txt_parse: bad arguments");
  char dl = (char)delimiter;
  auto cut = split_ranges(buf, len, nthreads);
  int T = (int)cut.size() - 1;
  std::vector<int64_t> L(T + 1, 0), R(T + 1, 0);
  run_threads(T, [&](int t) {
    int64_t lines = 0, rows = 0, nx;
    for (int64_t s = cut[t]; s < cut[t + 1]; s = nx) {
      int64_t e = line_end(buf, len, s, &nx);
      if (txt_fields(buf, s, e, dl, nullptr, 0) > 0) ++rows;
      ++lines;
    }
    L[t + 1] = lines, R[t + 1] = rows;
  });
  for (int t = 0; t < T; ++t) L[t + 1] += L[t], R[t + 1] += R[t];
  if (R[T] > 0 && (!out || !row_line))
    return dkm::fail(DKM_E_ARG, "txt_parse: NULL output");
  std::vector<Err> errs(T);
  run_threads(T, [&](int t) {
    int64_t line = L[t], row = R[t], nx;
    for (int64_t s = cut[t]; s < cut[t + 1]; s = nx, ++line) {
      int64_t e = line_end(buf, len, s, &nx);
      int64_t nf = txt_fields(buf, s, e, dl, out + row * n_cols, n_cols);
      if (nf == 0) continue;
      if (nf != n_cols) {
        errs[t].line = line;
        errs[t].msg = "Some errors were detected ! got " + std::to_string(nf) +
                      " columns instead of " + std::to_string(n_cols);
        return;
      }
      row_line[row++] = line;
    }
  });
  return report(errs);
}

}  // extern "C"
