// Spark 2.1 `libsvm` data source for one text file, host C++ (the input format of the
// reference's sample data, data/sample.txt, and of BASELINE config c1).
//
// Follows MLUtils.parseLibSVMFile / parseLibSVMRecord (spark-mllib 2.1.0, build.sbt:7-12):
//   lines are trimmed; empty lines and lines starting with '#' are skipped;
//   a record is "label index:value index:value ..." split on ' ' (empty items ignored);
//   indices are one-based in the file and become index - 1; they must be strictly ascending
//   ("indices should be one-based and in ascending order");
//   numFeatures (when not given) = max over rows of the row's last 0-based index, + 1, where an
//   empty row counts as index 0 (lastOption.getOrElse(0)).
// Numbers parse as Java's Double.parseDouble / Integer.parseInt would for decimal input
// (strtod is correctly rounded, like Java); trailing garbage in a token is an error.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/fm_hip.h"

namespace fmhip {
void set_error(const std::string& msg);
namespace {

struct ParseError {
  std::string msg;
};
#define FM_REQUIRE(cond, m)            \
  do {                                 \
    if (!(cond)) throw ParseError{(m)}; \
  } while (0)

struct Parsed {
  std::vector<double> label, val;
  std::vector<int64_t> row_ptr{0};
  std::vector<int32_t> col;
  int64_t max_last = 0;
};

inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v'; }

double parse_double(const std::string& tok, const std::string& line) {
  FM_REQUIRE(!tok.empty(), "libsvm: empty number in line \"" + line + "\"");
  char* end = nullptr;
  errno = 0;
  const double v = std::strtod(tok.c_str(), &end);
  FM_REQUIRE(end == tok.c_str() + tok.size(), "libsvm: bad number \"" + tok + "\" in line \"" + line + "\"");
  return v;
}

int64_t parse_int(const std::string& tok, const std::string& line) {
  FM_REQUIRE(!tok.empty(), "libsvm: empty index in line \"" + line + "\"");
  char* end = nullptr;
  errno = 0;
  const long long v = std::strtoll(tok.c_str(), &end, 10);
  FM_REQUIRE(end == tok.c_str() + tok.size() && errno == 0 && v >= INT32_MIN && v <= INT32_MAX,
             "libsvm: bad index \"" + tok + "\" in line \"" + line + "\"");
  return v;
}

void parse_file(const char* path, Parsed& out) {
  FILE* f = std::fopen(path, "rb");
  FM_REQUIRE(f != nullptr, std::string("libsvm: cannot open ") + path);
  std::string data;
  char buf[1 << 16];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, got);
  std::fclose(f);
  size_t pos = 0;
  while (pos < data.size()) {
    size_t eol = data.find('\n', pos);
    if (eol == std::string::npos) eol = data.size();
    size_t a = pos, b = eol;
    pos = eol + 1;
    while (a < b && is_space(data[a])) ++a;  // String.trim
    while (b > a && is_space(data[b - 1])) --b;
    if (a == b || data[a] == '#') continue;
    const std::string line = data.substr(a, b - a);
    // split(' '): items separated by single spaces, empty items dropped after the label
    std::vector<std::string> items;
    size_t s = 0;
    while (s <= line.size()) {
      size_t e = line.find(' ', s);
      if (e == std::string::npos) e = line.size();
      items.push_back(line.substr(s, e - s));
      s = e + 1;
    }
    out.label.push_back(parse_double(items[0], line));
    int64_t previous = -1, last = 0;
    for (size_t i = 1; i < items.size(); ++i) {
      if (items[i].empty()) continue;
      const size_t c = items[i].find(':');
      FM_REQUIRE(c != std::string::npos, "libsvm: item without ':' in line \"" + line + "\"");
      const int64_t index = parse_int(items[i].substr(0, c), line) - 1;
      const size_t c2 = items[i].find(':', c + 1);
      const double value = parse_double(items[i].substr(c + 1, c2 == std::string::npos ? std::string::npos : c2 - c - 1), line);
      FM_REQUIRE(index > previous, "libsvm: indices should be one-based and in ascending order; line \"" + line + "\"");
      previous = index;
      last = index;
      out.col.push_back((int32_t)index);
      out.val.push_back(value);
    }
    out.max_last = std::max(out.max_last, last);
    out.row_ptr.push_back((int64_t)out.col.size());
  }
}

}  // namespace
}  // namespace fmhip

using namespace fmhip;

extern "C" int fm_read_libsvm(const char* path, int64_t cap_rows, int64_t cap_nnz, double* label, int64_t* row_ptr,
                              int32_t* col, double* val, int64_t* n_rows, int64_t* nnz, int64_t* num_features) {
  try {
    FM_REQUIRE(path && n_rows && nnz && num_features, "null argument");
    Parsed p;
    parse_file(path, p);
    const int64_t B = (int64_t)p.label.size(), N = (int64_t)p.col.size();
    *n_rows = B;
    *nnz = N;
    *num_features = p.max_last + 1;
    if (cap_rows == 0 && cap_nnz == 0) return FM_OK;  // sizing call
    FM_REQUIRE(cap_rows >= B && cap_nnz >= N, "libsvm: output buffers too small");
    FM_REQUIRE(label && row_ptr && (N == 0 || (col && val)), "null output buffer");
    std::memcpy(label, p.label.data(), sizeof(double) * B);
    std::memcpy(row_ptr, p.row_ptr.data(), sizeof(int64_t) * (B + 1));
    if (N) {
      std::memcpy(col, p.col.data(), sizeof(int32_t) * N);
      std::memcpy(val, p.val.data(), sizeof(double) * N);
    }
    return FM_OK;
  } catch (const ParseError& e) {
    set_error(e.msg);
    return FM_ERR_ARG;
  } catch (const std::exception& e) {
    set_error(e.what());
    return FM_ERR_ARG;
  }
}
