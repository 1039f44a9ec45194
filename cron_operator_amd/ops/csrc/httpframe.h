// HTTP/1.1 framing helpers shared by the native extensions (`_httpcodec`, `_netconn`).
//
// Byte-level primitives only -- no Python objects -- so both the one-shot parsers of
// `_httpcodec` and the incremental connection parser of `_netconn` use one definition
// of whitespace, header-name matching and number parsing (the semantics of the
// pure-Python parsers in runtime/fasthttp.py that the tests use as the oracle).
#pragma once

#include <cstddef>
#include <cstring>

namespace httpframe {

// str.strip() of a latin-1 decoded string: ASCII whitespace, \x1c-\x1f, \x85, \xa0
inline bool is_space(unsigned char c) {
  return c == ' ' || (c >= '\t' && c <= '\r') || (c >= 0x1c && c <= 0x1f) || c == 0x85 || c == 0xa0;
}

// bytes.strip(): ASCII whitespace only
inline bool is_bytes_space(unsigned char c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

inline void strip(const unsigned char*& b, const unsigned char*& e) {
  while (b < e && is_space(*b)) ++b;
  while (e > b && is_space(e[-1])) --e;
}

inline unsigned char lower(unsigned char c) { return (c >= 'A' && c <= 'Z') ? c + 32 : c; }

inline bool ieq(const unsigned char* b, const unsigned char* e, const char* lit) {
  const size_t n = std::strlen(lit);
  if (static_cast<size_t>(e - b) != n) return false;
  for (size_t i = 0; i < n; ++i)
    if (lower(b[i]) != static_cast<unsigned char>(lit[i])) return false;
  return true;
}

inline bool icontains(const unsigned char* b, const unsigned char* e, const char* lit) {
  const size_t n = std::strlen(lit);
  for (const unsigned char* p = b; p + n <= e; ++p) {
    size_t i = 0;
    while (i < n && lower(p[i]) == static_cast<unsigned char>(lit[i])) ++i;
    if (i == n) return true;
  }
  return false;
}

inline const unsigned char* find(const unsigned char* b, const unsigned char* e, const char* lit, size_t n) {
  if (e < b || static_cast<size_t>(e - b) < n) return nullptr;
  return static_cast<const unsigned char*>(memmem(b, static_cast<size_t>(e - b), lit, n));
}

// Decimal integer with optional surrounding whitespace (int(v) for the values we accept)
inline bool parse_dec(const unsigned char* b, const unsigned char* e, long long* out) {
  strip(b, e);
  if (b == e) return false;
  long long v = 0;
  for (const unsigned char* p = b; p < e; ++p) {
    if (*p < '0' || *p > '9') return false;
    if (v > (1LL << 52)) return false;
    v = v * 10 + (*p - '0');
  }
  *out = v;
  return true;
}

inline bool parse_hex(const unsigned char* b, const unsigned char* e, long long* out) {
  strip(b, e);
  if (b == e) return false;
  long long v = 0;
  for (const unsigned char* p = b; p < e; ++p) {
    int d;
    if (*p >= '0' && *p <= '9') d = *p - '0';
    else if (*p >= 'a' && *p <= 'f') d = *p - 'a' + 10;
    else if (*p >= 'A' && *p <= 'F') d = *p - 'A' + 10;
    else return false;
    if (v > (1LL << 48)) return false;
    v = v * 16 + d;
  }
  *out = v;
  return true;
}

// The size of the chunk whose size line is [b, nl) (extensions after ';' ignored).
inline bool chunk_size(const unsigned char* b, const unsigned char* nl, long long* out) {
  const unsigned char* semi = static_cast<const unsigned char*>(memchr(b, ';', static_cast<size_t>(nl - b)));
  return parse_hex(b, semi ? semi : nl, out);
}

// A response head [b, hend) (hend at the blank line's CRLFCRLF).  Framing fields only.
struct ResponseHead {
  long long status = 0;
  long long content_length = -1;  // -1: absent
  long long retry_after = -1;     // -1: absent or not a number
  bool chunked = false;
  bool close = false;             // HTTP/1.0 without keep-alive, or Connection: close
};

// false: malformed status line or Content-Length
inline bool parse_response_head(const unsigned char* b, const unsigned char* hend, ResponseHead* h) {
  const unsigned char* l_end = find(b, hend + 2, "\r\n", 2);
  if (!l_end) return false;
  const unsigned char* sp1 = static_cast<const unsigned char*>(memchr(b, ' ', static_cast<size_t>(l_end - b)));
  if (!sp1) return false;
  const unsigned char* sp2 =
      static_cast<const unsigned char*>(memchr(sp1 + 1, ' ', static_cast<size_t>(l_end - sp1 - 1)));
  if (!parse_dec(sp1 + 1, sp2 ? sp2 : l_end, &h->status)) return false;
  h->close = (sp1 - b) == 8 && std::memcmp(b, "HTTP/1.0", 8) == 0;
  const unsigned char* p = l_end + 2;
  while (p < hend + 2) {
    const unsigned char* nl = find(p, hend + 2, "\r\n", 2);
    if (!nl) break;
    const unsigned char* colon = static_cast<const unsigned char*>(memchr(p, ':', static_cast<size_t>(nl - p)));
    const unsigned char *kb = p, *ke = colon ? colon : nl;
    const unsigned char *vb = colon ? colon + 1 : nl, *ve = nl;
    strip(kb, ke);
    strip(vb, ve);
    if (ieq(kb, ke, "content-length")) {
      if (!parse_dec(vb, ve, &h->content_length)) return false;
    } else if (ieq(kb, ke, "transfer-encoding")) {
      h->chunked = icontains(vb, ve, "chunked");
    } else if (ieq(kb, ke, "connection")) {
      if (ieq(vb, ve, "close")) h->close = true;
      else if (ieq(vb, ve, "keep-alive")) h->close = false;
    } else if (ieq(kb, ke, "retry-after")) {
      long long ra;
      h->retry_after = parse_dec(vb, ve, &ra) ? ra : -1;
    }
    p = nl + 2;
  }
  return true;
}

}  // namespace httpframe
