// Layer-tar walk: walker.LayerTar.Walk (pkg/fanal/walker/tar.go:35-103) with
// the tar reading Go's archive/tar does for it (Reader.Next: ustar / GNU /
// PAX headers, checksum, GNU long names, PAX path and size records), over a
// tar held in memory.  Only what Walk consumes is produced: the cleaned path,
// content offset and size of every regular file it would analyze, and the
// opaque-directory and whiteout lists it returns.
#include "tar.h"

#include <algorithm>
#include <cstring>

namespace tsg {
namespace {

constexpr size_t kBlock = 512;

bool all_zero(const uint8_t* b) {
  for (size_t i = 0; i < kBlock; ++i) if (b[i]) return false;
  return true;
}

// NUL-terminated field
std::string field(const uint8_t* b, size_t n) {
  size_t e = 0;
  while (e < n && b[e]) ++e;
  return std::string(reinterpret_cast<const char*>(b), e);
}

// archive/tar parseNumeric: base-256 when the high bit of the first byte is
// set, else octal with leading / trailing spaces and NULs trimmed
bool parse_numeric(const uint8_t* b, size_t n, int64_t* out) {
  if (n > 0 && (b[0] & 0x80)) {
    const uint8_t inv = (b[0] & 0x40) ? 0xff : 0x00;   // negative numbers are two's complement
    uint64_t x = 0;
    for (size_t i = 0; i < n; ++i) {
      uint8_t c = b[i] ^ inv;
      if (i == 0) c &= 0x7f;
      if ((x >> 56) != 0) return false;                // overflow
      x = (x << 8) | c;
    }
    if (x >> 63) return false;
    *out = inv ? ~static_cast<int64_t>(x) : static_cast<int64_t>(x);
    return true;
  }
  size_t s = 0, e = n;
  while (s < e && (b[s] == ' ' || b[s] == 0)) ++s;
  while (e > s && (b[e - 1] == ' ' || b[e - 1] == 0)) --e;
  int64_t x = 0;
  if (s == e) { *out = 0; return true; }
  for (size_t i = s; i < e; ++i) {
    if (b[i] < '0' || b[i] > '7') return false;
    if (x > (INT64_MAX >> 3)) return false;
    x = x * 8 + (b[i] - '0');
  }
  *out = x;
  return true;
}

// header checksum: sum of the block with the checksum field read as spaces,
// unsigned or signed bytes (archive/tar format.go computeChecksum)
bool checksum_ok(const uint8_t* h) {
  int64_t want = 0;
  if (!parse_numeric(h + 148, 8, &want)) return false;
  int64_t u = 0, sg = 0;
  for (size_t i = 0; i < kBlock; ++i) {
    const uint8_t c = (i >= 148 && i < 156) ? ' ' : h[i];
    u += c;
    sg += static_cast<int8_t>(c);
  }
  return want == u || want == sg;
}

// PAX records "%d %s=%s\n" (archive/tar parsePAXRecord); only path and size
// matter to the walk
bool parse_pax(const uint8_t* p, size_t n, std::string* path, bool* has_path, int64_t* size, bool* has_size) {
  size_t i = 0;
  while (i < n) {
    size_t sp = i;
    while (sp < n && p[sp] != ' ') ++sp;
    if (sp >= n) return false;
    int64_t len = 0;
    for (size_t k = i; k < sp; ++k) {
      if (p[k] < '0' || p[k] > '9') return false;
      len = len * 10 + (p[k] - '0');
      if (len > static_cast<int64_t>(n)) return false;
    }
    if (len <= static_cast<int64_t>(sp - i) || i + static_cast<size_t>(len) > n) return false;
    const size_t end = i + static_cast<size_t>(len);
    if (p[end - 1] != '\n') return false;
    const std::string rec(reinterpret_cast<const char*>(p + sp + 1), end - 1 - (sp + 1));
    const size_t eq = rec.find('=');
    if (eq == std::string::npos) return false;
    const std::string key = rec.substr(0, eq), val = rec.substr(eq + 1);
    // validPAXRecord: a non-empty key; no NUL in the value of path, linkpath,
    // uname or gname, nor in the key of any other record
    if (key.empty()) return false;
    const bool value_checked = key == "path" || key == "linkpath" || key == "uname" || key == "gname";
    if ((value_checked ? val : key).find('\0') != std::string::npos) return false;
    if (key == "path") { *path = val; *has_path = true; }
    else if (key == "size") {
      // strconv.ParseInt(v, 10, 64): optional sign, decimal digits, range
      // checked; a negative size is rejected later (handleRegularFile)
      size_t k = 0;
      bool neg = false;
      if (k < val.size() && (val[k] == '+' || val[k] == '-')) neg = val[k++] == '-';
      if (k == val.size()) return false;
      int64_t v = 0;
      for (; k < val.size(); ++k) {
        const char c = val[k];
        if (c < '0' || c > '9') return false;
        if (v > (INT64_MAX - (c - '0')) / 10) return false;   // out of range: ErrHeader
        v = v * 10 + (c - '0');
      }
      *size = neg ? -v : v;
      *has_size = true;
    }
    i = end;
  }
  return true;
}

// path.Split
void go_path_split(const std::string& p, std::string* dir, std::string* file) {
  const size_t i = p.rfind('/');
  *dir = i == std::string::npos ? "" : p.substr(0, i + 1);
  *file = i == std::string::npos ? p : p.substr(i + 1);
}

std::string trim_left_slash(const std::string& s) {
  size_t i = 0;
  while (i < s.size() && s[i] == '/') ++i;
  return s.substr(i);
}

// filepath.Rel(base, targ) for two relative, cleaned paths; only whether the
// result starts with "../" matters to underSkippedDir (tar.go:107-119)
bool rel_escapes(const std::string& base, const std::string& targ) {
  if (base == ".") return targ == ".." || targ.rfind("../", 0) == 0;
  if (targ == base) return false;
  if (targ.size() > base.size() && targ.compare(0, base.size(), base) == 0 && targ[base.size()] == '/') return false;
  return true;
}

// ---- doublestar ----------------------------------------------------------

bool class_match(const std::string& p, size_t* i, char c, bool* ok) {
  // p[*i] == '['; on return *i is past ']'
  size_t k = *i + 1;
  bool neg = false;
  if (k < p.size() && (p[k] == '!' || p[k] == '^')) { neg = true; ++k; }
  bool hit = false, first = true;
  while (k < p.size() && (p[k] != ']' || first)) {
    first = false;
    char lo = p[k];
    if (lo == '\\') { if (++k >= p.size()) { *ok = false; return false; } lo = p[k]; }
    char hi = lo;
    if (k + 2 < p.size() && p[k + 1] == '-' && p[k + 2] != ']') {
      k += 2;
      hi = p[k];
      if (hi == '\\') { if (++k >= p.size()) { *ok = false; return false; } hi = p[k]; }
    }
    if (lo <= c && c <= hi) hit = true;
    ++k;
  }
  if (k >= p.size()) { *ok = false; return false; }   // no closing ']'
  *i = k + 1;
  return hit != neg;
}

// one path component against a brace-free component pattern
bool comp_match(const std::string& p, size_t pi, const std::string& s, size_t si, bool* ok) {
  while (pi < p.size()) {
    const char c = p[pi];
    if (c == '*') {
      while (pi < p.size() && p[pi] == '*') ++pi;
      if (pi == p.size()) return true;
      for (size_t k = si; k <= s.size(); ++k) {
        if (comp_match(p, pi, s, k, ok)) return true;
        if (!*ok) return false;
      }
      return false;
    }
    if (si >= s.size()) {
      // validate the rest of the pattern for a bad-pattern error
      if (c == '[') { size_t j = pi; class_match(p, &j, 0, ok); }
      return false;
    }
    if (c == '?') { ++pi; ++si; continue; }
    if (c == '[') {
      if (!class_match(p, &pi, s[si], ok)) return false;
      ++si;
      continue;
    }
    char lit = c;
    if (c == '\\') {
      if (pi + 1 >= p.size()) { *ok = false; return false; }
      lit = p[++pi];
    }
    if (lit != s[si]) return false;
    ++pi;
    ++si;
  }
  return si == s.size();
}

std::vector<std::string> split_slash(const std::string& s) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    const size_t e = s.find('/', b);
    out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) break;
    b = e + 1;
  }
  return out;
}

bool comps_match(const std::vector<std::string>& p, size_t pi, const std::vector<std::string>& n, size_t ni, bool* ok) {
  if (pi == p.size()) return ni == n.size();
  if (p[pi] == "**") {
    for (size_t k = ni; k <= n.size(); ++k) {
      if (comps_match(p, pi + 1, n, k, ok)) return true;
      if (!*ok) return false;
    }
    return false;
  }
  if (ni == n.size()) return false;
  if (!comp_match(p[pi], 0, n[ni], 0, ok)) return false;
  return comps_match(p, pi + 1, n, ni + 1, ok);
}

// expand the first top-level {a,b,...} (recursively) into brace-free patterns
bool expand_braces(const std::string& p, std::vector<std::string>* out, int depth = 0) {
  if (depth > 16 || out->size() > 4096) return false;
  size_t open = std::string::npos;
  for (size_t i = 0; i < p.size(); ++i) {
    if (p[i] == '\\') { ++i; continue; }
    if (p[i] == '{') { open = i; break; }
  }
  if (open == std::string::npos) { out->push_back(p); return true; }
  int d = 0;
  std::vector<size_t> commas;
  size_t close = std::string::npos;
  for (size_t i = open; i < p.size(); ++i) {
    if (p[i] == '\\') { ++i; continue; }
    if (p[i] == '{') ++d;
    else if (p[i] == '}') { if (--d == 0) { close = i; break; } }
    else if (p[i] == ',' && d == 1) commas.push_back(i);
  }
  if (close == std::string::npos) return false;          // unclosed brace: bad pattern
  size_t b = open + 1;
  commas.push_back(close);
  for (size_t c : commas) {
    if (!expand_braces(p.substr(0, open) + p.substr(b, c - b) + p.substr(close + 1), out, depth + 1)) return false;
    b = c + 1;
  }
  return true;
}

}  // namespace

std::string go_path_clean(const std::string& p) {
  if (p.empty()) return ".";
  const bool rooted = p[0] == '/';
  std::vector<std::string> parts;
  size_t i = 0;
  while (i < p.size()) {
    while (i < p.size() && p[i] == '/') ++i;
    size_t e = i;
    while (e < p.size() && p[e] != '/') ++e;
    const std::string seg = p.substr(i, e - i);
    i = e;
    if (seg.empty() || seg == ".") continue;
    if (seg == "..") {
      if (!parts.empty() && parts.back() != "..") parts.pop_back();
      else if (!rooted) parts.push_back("..");
      continue;
    }
    parts.push_back(seg);
  }
  std::string out = rooted ? "/" : "";
  for (size_t k = 0; k < parts.size(); ++k) {
    if (k) out += '/';
    out += parts[k];
  }
  return out.empty() ? "." : out;
}

bool doublestar_match(const std::string& pattern, const std::string& name) {
  std::vector<std::string> alts;
  if (!expand_braces(pattern, &alts)) return false;
  const std::vector<std::string> n = split_slash(name);
  for (const std::string& a : alts) {
    bool ok = true;
    const bool m = comps_match(split_slash(a), 0, n, 0, &ok);
    if (!ok) return false;                                // bad pattern: SkipPath returns false
    if (m) return true;
  }
  return false;
}

bool TarInput::skip(uint64_t n, uint64_t* got, std::string* err) {
  uint8_t buf[16384];
  *got = 0;
  while (*got < n) {
    size_t g = 0;
    if (!read(buf, static_cast<size_t>(std::min<uint64_t>(sizeof(buf), n - *got)), &g, err)) return false;
    if (g == 0) break;
    *got += g;
  }
  return true;
}

bool read_full(TarInput& in, uint8_t* dst, size_t n, size_t* got, std::string* err) {
  *got = 0;
  while (*got < n) {
    size_t g = 0;
    if (!in.read(dst + *got, n - *got, &g, err)) return false;
    if (g == 0) break;
    *got += g;
  }
  return true;
}

bool MemTarInput::read(uint8_t* dst, size_t n, size_t* got, std::string*) {
  const size_t k = static_cast<size_t>(std::min<uint64_t>(n, n_ - pos));
  std::memcpy(dst, p_ + pos, k);
  pos += k;
  *got = k;
  return true;
}

bool MemTarInput::skip(uint64_t n, uint64_t* got, std::string*) {
  *got = std::min<uint64_t>(n, n_ - pos);
  pos += *got;
  return true;
}

bool walk_layer(TarInput& in, const std::vector<std::string>& skip_files_in, const std::vector<std::string>& skip_dirs_in,
                LayerWalk* out, const TarFileFn& on_file, std::string* err) {
  auto clean_skip = [](const std::vector<std::string>& v) {   // utils.CleanSkipPaths
    std::vector<std::string> r;
    for (const auto& s : v) r.push_back(trim_left_slash(go_path_clean(s)));
    return r;
  };
  auto skip_path = [](const std::string& path, const std::vector<std::string>& pats) {   // utils.SkipPath
    const std::string p = trim_left_slash(path);
    for (const auto& pat : pats) if (doublestar_match(pat, p)) return true;
    return false;
  };
  const std::vector<std::string> skip_files = clean_skip(skip_files_in), skip_dirs = clean_skip(skip_dirs_in);
  std::vector<std::string> skipped_dirs;
  auto fail = [&](const char* what) {
    *err = std::string("failed to extract the archive: archive/tar: ") + what;
    return false;
  };
  // the data of the entry just read (size bytes) plus its block padding
  auto skip_data = [&](uint64_t n) {
    uint64_t got = 0;
    if (!in.skip(n, &got, err)) return false;
    if (got < n) return fail("unexpected EOF");
    return true;
  };
  constexpr uint64_t kMaxSpecialFileSize = 1 << 20;           // archive/tar maxSpecialFileSize
  uint8_t h[kBlock];
  std::vector<uint8_t> special;
  std::string long_name, pax_path;
  bool has_long = false, has_pax_path = false, has_pax_size = false;
  int64_t pax_size = 0;
  for (;;) {
    size_t got = 0;
    if (!read_full(in, h, kBlock, &got, err)) return false;
    if (got == 0) return true;                                 // io.EOF at a block boundary
    if (got < kBlock) return fail("unexpected EOF");
    if (all_zero(h)) {
      // end of archive: a second zero block (or the end of the data) must follow
      uint8_t h2[kBlock];
      if (!read_full(in, h2, kBlock, &got, err)) return false;
      if (got == kBlock && !all_zero(h2)) return fail("invalid tar header");
      return true;
    }
    if (!checksum_ok(h)) return fail("invalid tar header");
    int64_t size = 0;
    const char type = static_cast<char>(h[156]);
    // the raw header's size goes through handleRegularFile before any PAX
    // record applies: negative is ErrHeader unless the type carries no data
    const bool raw_header_only = type == '1' || type == '2' || type == '3' || type == '4' || type == '5' || type == '6';
    if (!parse_numeric(h + 124, 12, &size)) return fail("invalid tar header");
    if (size < 0) {
      if (!raw_header_only) return fail("invalid tar header");
      size = 0;
    }
    const bool ustar = std::memcmp(h + 257, "ustar", 5) == 0;
    std::string name = field(h, 100);
    if (ustar && std::memcmp(h + 257, "ustar\0" "00", 8) == 0) {
      const std::string prefix = field(h + 345, 155);       // POSIX ustar prefix
      if (!prefix.empty()) name = prefix + "/" + name;
    }
    const uint64_t padded = (static_cast<uint64_t>(size) + kBlock - 1) / kBlock * kBlock;
    if (type == 'x' || type == 'g' || type == 'L' || type == 'K') {
      // readSpecialFile: at most 1 MiB, read whole (a shorter archive is an unexpected EOF)
      if (static_cast<uint64_t>(size) > kMaxSpecialFileSize) return fail("header field too long");
      special.resize(static_cast<size_t>(size));
      if (!read_full(in, special.data(), special.size(), &got, err)) return false;
      if (got < special.size()) return fail("unexpected EOF");
      if (!skip_data(padded - static_cast<uint64_t>(size))) return false;
      const uint8_t* d = special.data();
      if (type == 'x') {
        if (!parse_pax(d, static_cast<size_t>(size), &pax_path, &has_pax_path, &pax_size, &has_pax_size))
          return fail("invalid tar header");
      } else if (type == 'L') {
        long_name = field(d, static_cast<size_t>(size));
        has_long = true;
      }
      // 'g' (global PAX) is returned by Next as its own entry: Walk skips it
      // (default case); 'K' (GNU long link name) only affects Linkname
      continue;
    }
    if (has_long) name = long_name;
    if (has_pax_path) name = pax_path;
    if (has_pax_size) size = pax_size;
    has_long = has_pax_path = has_pax_size = false;
    char tf = type;
    // Reader.Next: TypeRegA ('\0') becomes TypeDir for names ending in '/', else TypeReg
    if (tf == '\0') tf = (!name.empty() && name.back() == '/') ? '5' : '0';
    // Reader.handleRegularFile: header-only types (links, devices, dirs,
    // fifos) consume no data whatever their size field says
    const bool has_data = !(tf == '1' || tf == '2' || tf == '3' || tf == '4' || tf == '5' || tf == '6');
    if (has_data && size < 0) return fail("invalid tar header");   // handleRegularFile: Size < 0 is ErrHeader
    const uint64_t data_bytes = has_data ? static_cast<uint64_t>(size) : 0;
    const uint64_t data_padded = has_data ? (data_bytes + kBlock - 1) / kBlock * kBlock : 0;
    if (data_padded < data_bytes) return fail("invalid tar header");   // size near 2^64: no padded length
    // ---- walker.LayerTar.Walk (tar.go:46-90)
    std::string file_path = trim_left_slash(go_path_clean(name));
    std::string dir, fname;
    go_path_split(file_path, &dir, &fname);
    bool hand = false;
    if (fname == ".wh..wh..opq") {
      out->opq_dirs.push_back(dir);
    } else if (fname.rfind(".wh.", 0) == 0) {
      out->wh_files.push_back(go_path_clean(dir + fname.substr(4)));   // path.Join(fileDir, name)
    } else if (tf == '5') {
      if (skip_path(file_path, skip_dirs)) skipped_dirs.push_back(file_path);
      // a directory reaches AnalyzeFile, which returns at IsDir
    } else if (tf == '0' && !skip_path(file_path, skip_files)) {   // TypeReg; others: Walk's default
      hand = true;
      for (const auto& sd : skipped_dirs) if (!rel_escapes(sd, file_path)) { hand = false; break; }
    }
    uint64_t consumed = 0;
    if (hand) {
      out->files.push_back(TarFile{file_path, in.pos, data_bytes});
      const uint64_t p0 = in.pos;
      if (on_file && !on_file(file_path, data_bytes, in, err)) return false;
      consumed = in.pos - p0;
      if (consumed > data_bytes) { *err = "internal: file reader overran its entry"; return false; }
    }
    if (!skip_data(data_padded - consumed)) return false;
  }
}

bool walk_layer_tar(const uint8_t* tar, size_t len, const std::vector<std::string>& skip_files,
                    const std::vector<std::string>& skip_dirs, LayerWalk* out, std::string* err) {
  MemTarInput in(tar, len);
  return walk_layer(in, skip_files, skip_dirs, out, nullptr, err);
}

}  // namespace tsg
