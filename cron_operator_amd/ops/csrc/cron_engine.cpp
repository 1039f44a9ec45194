// Native cron next-fire engine (CPython extension `_cron_engine`).
//
// Native twin of cron_operator_amd/cron/{parser,schedule}.py.  It implements the
// behaviour the reference gets from robfig/cron/v3 ParseStandard + Schedule.Next
// (reference: internal/controller/cron_controller.go:389-437, HOT LOOP 3), plus
// a bulk "missed runs" scan that counts missed ticks by whole days when the
// schedule's zone has a constant offset over the scanned span, instead of
// walking every tick (the reference walks every tick: O(#missed)).
//
// Time model: Go time.Time semantics over (unix seconds, nanoseconds, zone).
// Zones are IANA TZif v2+ blobs handed in from Python (the tzdata wheel); the
// POSIX TZ footer extends the transition table into the future.
//
// Exposed (see ops/cron_native.py for the Python-facing wrapper):
//   register_zone(name:str, tzif:bytes) -> int      zone id (0 = UTC)
//   register_fixed_zone(name:str, offset:int) -> int
//   zone_offset(zone:int, unix:int) -> int
//   parse(spec:str) -> Schedule | raises ValueError(<robfig message>)
//   Schedule.next(sec, nsec, zone) -> (sec, nsec)   (zero time = (ZERO_UNIX, 0))
//   Schedule.missed(e_sec, e_nsec, n_sec, n_nsec, zone) -> (last_sec, last_nsec, count, unschedulable)
//   Schedule.masks() -> (sec, min, hour, dom, month, dow, zone)  (zone -1 = Local)
//   Schedule.is_every / Schedule.delay
//   bulk_next(schedules:list, secs:list, nsecs:list, zone) -> list[(sec, nsec)]

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int64_t kNanos = 1000000000LL;
constexpr int64_t kUnixToAbs = 62135596800LL;
constexpr int64_t kZeroUnix = -kUnixToAbs;
constexpr uint64_t kStarBit = 1ULL << 63;

// ------------------------------------------------------------------ civil calendar

inline int64_t floordiv(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) --q;
  return q;
}
inline int64_t floormod(int64_t a, int64_t b) { return a - floordiv(a, b) * b; }

// days since 1970-01-01; month may be out of 1..12, day may be out of range.
int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
  y += floordiv(m - 1, 12);
  m = floormod(m - 1, 12) + 1;
  const int64_t yy = y - (m <= 2 ? 1 : 0);
  const int64_t era = floordiv(yy, 400);
  const int64_t yoe = yy - era * 400;
  const int64_t mp = m > 2 ? m - 3 : m + 9;
  const int64_t doy = (153 * mp + 2) / 5;
  const int64_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468 + (d - 1);
}

struct Civil {
  int64_t y;
  int m, d;
};

Civil civil_from_days(int64_t z) {
  z += 719468;
  const int64_t era = floordiv(z, 146097);
  const int64_t doe = z - era * 146097;
  const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const int64_t mp = (5 * doy + 2) / 153;
  const int d = static_cast<int>(doy - (153 * mp + 2) / 5 + 1);
  const int m = static_cast<int>(mp < 10 ? mp + 3 : mp - 9);
  return Civil{yoe + era * 400 + (m <= 2 ? 1 : 0), m, d};
}

inline bool is_leap(int64_t y) { return (y % 4 == 0 && y % 100 != 0) || y % 400 == 0; }
inline int days_in_month(int64_t y, int m) {
  static const int kDays[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
  return (m == 2 && is_leap(y)) ? 29 : kDays[m - 1];
}

// ------------------------------------------------------------------ zones

struct PosixRule {
  // kind: 0 = Julian (J n, 1..365, no leap day), 1 = zero-based day (n, 0..365), 2 = Mm.w.d
  int kind = 2;
  int day = 0, week = 0, mon = 0;
  int64_t time = 7200;  // seconds after local midnight
};

struct PosixTZ {
  bool valid = false;
  int64_t std_off = 0;  // seconds east of UTC
  bool has_dst = false;
  int64_t dst_off = 0;
  PosixRule start, end;
};

struct Zone {
  std::string name;
  bool fixed = true;
  int64_t fixed_off = 0;
  std::vector<int64_t> trans;    // transition instants (unix seconds)
  std::vector<int32_t> trans_off;  // offset in effect from trans[i]
  int64_t first_off = 0;           // offset before the first transition
  PosixTZ footer;
};

std::mutex g_zone_mu;
std::vector<std::shared_ptr<Zone>> g_zones;  // index = zone id

// -- POSIX TZ parsing (RFC 8536 section 3.3 / POSIX.1 TZ) -------------------------

bool parse_name(const char*& p) {
  if (*p == '<') {
    ++p;
    while (*p && *p != '>') ++p;
    if (*p != '>') return false;
    ++p;
    return true;
  }
  const char* s = p;
  while (*p && ((*p >= 'a' && *p <= 'z') || (*p >= 'A' && *p <= 'Z'))) ++p;
  return p - s >= 3;
}

bool parse_num(const char*& p, int64_t* out) {
  if (!(*p >= '0' && *p <= '9')) return false;
  int64_t v = 0;
  while (*p >= '0' && *p <= '9') v = v * 10 + (*p++ - '0');
  *out = v;
  return true;
}

// [+-]hh[:mm[:ss]] -> seconds (sign as written)
bool parse_hms(const char*& p, int64_t* out) {
  int sign = 1;
  if (*p == '+') {
    ++p;
  } else if (*p == '-') {
    sign = -1;
    ++p;
  }
  int64_t h = 0, m = 0, s = 0;
  if (!parse_num(p, &h)) return false;
  if (*p == ':') {
    ++p;
    if (!parse_num(p, &m)) return false;
    if (*p == ':') {
      ++p;
      if (!parse_num(p, &s)) return false;
    }
  }
  *out = sign * (h * 3600 + m * 60 + s);
  return true;
}

bool parse_rule(const char*& p, PosixRule* r) {
  int64_t v = 0;
  if (*p == 'J') {
    ++p;
    if (!parse_num(p, &v)) return false;
    r->kind = 0;
    r->day = static_cast<int>(v);
  } else if (*p == 'M') {
    ++p;
    int64_t mon = 0, wk = 0, dd = 0;
    if (!parse_num(p, &mon) || *p++ != '.') return false;
    if (!parse_num(p, &wk) || *p++ != '.') return false;
    if (!parse_num(p, &dd)) return false;
    r->kind = 2;
    r->mon = static_cast<int>(mon);
    r->week = static_cast<int>(wk);
    r->day = static_cast<int>(dd);
  } else {
    if (!parse_num(p, &v)) return false;
    r->kind = 1;
    r->day = static_cast<int>(v);
  }
  r->time = 7200;
  if (*p == '/') {
    ++p;
    if (!parse_hms(p, &r->time)) return false;
  }
  return true;
}

PosixTZ parse_posix(const std::string& s) {
  PosixTZ tz;
  const char* p = s.c_str();
  if (!*p) return tz;
  if (!parse_name(p)) return tz;
  int64_t off = 0;
  if (!parse_hms(p, &off)) return tz;
  tz.std_off = -off;  // POSIX offsets are west-positive
  if (!*p) {
    tz.valid = true;
    return tz;
  }
  if (!parse_name(p)) return tz;
  tz.has_dst = true;
  tz.dst_off = tz.std_off + 3600;
  if (*p && *p != ',') {
    if (!parse_hms(p, &off)) return tz;
    tz.dst_off = -off;
  }
  if (!*p) {  // no rule: US default
    tz.start = PosixRule{2, 0, 2, 3, 7200};
    tz.end = PosixRule{2, 0, 1, 11, 7200};
    tz.valid = true;
    return tz;
  }
  if (*p != ',') return tz;
  ++p;
  if (!parse_rule(p, &tz.start)) return tz;
  if (*p != ',') return tz;
  ++p;
  if (!parse_rule(p, &tz.end)) return tz;
  tz.valid = (*p == 0);
  return tz;
}

// Seconds from the start of year `y` (local midnight Jan 1) to the rule's day at 00:00.
int64_t rule_day_start(int64_t y, const PosixRule& r) {
  int64_t yday = 0;
  switch (r.kind) {
    case 0: {  // Jn: 1..365, Feb 29 never counted
      yday = r.day - 1;
      if (is_leap(y) && r.day >= 60) yday += 1;
      break;
    }
    case 1:
      yday = r.day;
      break;
    default: {
      const int64_t first = days_from_civil(y, r.mon, 1);
      const int64_t wd_first = floormod(first + 4, 7);  // 0 = Sunday
      int64_t d = floormod(r.day - wd_first, 7);           // first matching weekday (0-based day in month)
      d += static_cast<int64_t>(r.week - 1) * 7;
      const int dim = days_in_month(y, r.mon);
      while (d >= dim) d -= 7;
      yday = (first - days_from_civil(y, 1, 1)) + d;
      break;
    }
  }
  return yday * 86400;
}

int64_t posix_offset(const PosixTZ& tz, int64_t unix) {
  if (!tz.has_dst) return tz.std_off;
  // local standard year of the instant
  const int64_t local = unix + tz.std_off;
  const int64_t y = civil_from_days(floordiv(local, 86400)).y;
  auto in_dst = [&](int64_t yy) -> int {
    const int64_t ystart = days_from_civil(yy, 1, 1) * 86400;
    // start transition given in local standard time, end in local daylight time
    const int64_t s = ystart + rule_day_start(yy, tz.start) + tz.start.time - tz.std_off;
    const int64_t e = ystart + rule_day_start(yy, tz.end) + tz.end.time - tz.dst_off;
    if (s < e) return (unix >= s && unix < e) ? 1 : 0;
    // southern hemisphere: DST spans the new year
    return (unix >= e && unix < s) ? 0 : 1;
  };
  // Near a year boundary the transition of the neighbouring year may apply; the
  // in-year evaluation is exact for all real-world rules (transitions are far from
  // Jan 1), so a single evaluation suffices.
  return in_dst(y) ? tz.dst_off : tz.std_off;
}

int64_t zone_offset_at(const Zone& z, int64_t unix) {
  if (z.fixed) return z.fixed_off;
  if (z.trans.empty() || unix < z.trans.front()) {
    if (z.trans.empty() && z.footer.valid) return posix_offset(z.footer, unix);
    return z.first_off;
  }
  if (unix >= z.trans.back() && z.footer.valid) {
    // The footer governs instants after the last transition.  The last table entry
    // is still authoritative until the footer's next transition; evaluating the
    // footer directly gives the same answer for well-formed files.
    return posix_offset(z.footer, unix);
  }
  auto it = std::upper_bound(z.trans.begin(), z.trans.end(), unix);
  const size_t idx = static_cast<size_t>(it - z.trans.begin()) - 1;
  return z.trans_off[idx];
}

// Does the zone have a constant offset over [a, b]?
bool zone_constant_between(const Zone& z, int64_t a, int64_t b) {
  if (z.fixed) return true;
  const int64_t oa = zone_offset_at(z, a);
  if (zone_offset_at(z, b) != oa) return false;
  if (!z.trans.empty() && a < z.trans.back()) {
    auto it = std::upper_bound(z.trans.begin(), z.trans.end(), a);
    if (it != z.trans.end() && *it <= b) return false;
  }
  if (z.footer.valid && z.footer.has_dst && b >= (z.trans.empty() ? a : std::max(a, z.trans.back()))) {
    // footer DST: constant only if the span stays within one DST/STD run; sample daily
    for (int64_t t = a; t <= b; t += 86400) {
      if (posix_offset(z.footer, t) != oa) return false;
    }
  }
  return true;
}

inline uint32_t rd_be32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | uint32_t(p[3]);
}
inline int64_t rd_be64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return static_cast<int64_t>(v);
}

bool parse_tzif(const uint8_t* data, size_t n, Zone* z, std::string* err) {
  auto hdr_ok = [&](size_t off) { return off + 44 <= n && std::memcmp(data + off, "TZif", 4) == 0; };
  if (!hdr_ok(0)) {
    *err = "not a TZif file";
    return false;
  }
  const uint8_t version = data[4];
  auto counts = [&](size_t off, uint32_t c[6]) {
    for (int i = 0; i < 6; ++i) c[i] = rd_be32(data + off + 20 + 4 * i);
  };
  uint32_t c1[6];  // isutcnt, isstdcnt, leapcnt, timecnt, typecnt, charcnt
  counts(0, c1);
  size_t v1len = size_t(c1[3]) * 5 + size_t(c1[4]) * 6 + c1[5] + size_t(c1[2]) * 8 + c1[1] + c1[0];
  size_t off = 44;
  int tsize = 4;
  uint32_t c[6];
  std::memcpy(c, c1, sizeof c);
  if (version >= '2') {
    off = 44 + v1len;
    if (!hdr_ok(off)) {
      *err = "bad v2 header";
      return false;
    }
    counts(off, c);
    off += 44;
    tsize = 8;
  }
  const uint32_t isutcnt = c[0], isstdcnt = c[1], leapcnt = c[2], timecnt = c[3], typecnt = c[4],
                 charcnt = c[5];
  const size_t need = size_t(timecnt) * tsize + timecnt + size_t(typecnt) * 6 + charcnt +
                      size_t(leapcnt) * (tsize + 4) + isstdcnt + isutcnt;
  if (off + need > n || typecnt == 0) {
    *err = "truncated TZif data";
    return false;
  }
  const uint8_t* p = data + off;
  std::vector<int64_t> tt(timecnt);
  for (uint32_t i = 0; i < timecnt; ++i) {
    tt[i] = tsize == 8 ? rd_be64(p + 8 * i) : static_cast<int32_t>(rd_be32(p + 4 * i));
  }
  p += size_t(timecnt) * tsize;
  std::vector<uint8_t> idx(p, p + timecnt);
  p += timecnt;
  std::vector<int32_t> utoff(typecnt);
  std::vector<uint8_t> isdst(typecnt);
  for (uint32_t i = 0; i < typecnt; ++i) {
    utoff[i] = static_cast<int32_t>(rd_be32(p + 6 * i));
    isdst[i] = p[6 * i + 4];
  }
  p += size_t(typecnt) * 6 + charcnt + size_t(leapcnt) * (tsize + 4) + isstdcnt + isutcnt;
  z->trans.clear();
  z->trans_off.clear();
  for (uint32_t i = 0; i < timecnt; ++i) {
    if (idx[i] >= typecnt) {
      *err = "bad transition type index";
      return false;
    }
    z->trans.push_back(tt[i]);
    z->trans_off.push_back(utoff[idx[i]]);
  }
  // Offset before the first transition: first non-DST type (Go's lookupFirstZone heuristic)
  z->first_off = utoff[0];
  if (timecnt > 0 && isdst[idx[0]]) {
    for (uint32_t i = 0; i < typecnt; ++i) {
      if (!isdst[i]) {
        z->first_off = utoff[i];
        break;
      }
    }
  }
  if (version >= '2') {
    const size_t foot_off = static_cast<size_t>(p - data);
    if (foot_off < n && data[foot_off] == '\n') {
      size_t e = foot_off + 1;
      while (e < n && data[e] != '\n') ++e;
      z->footer = parse_posix(std::string(reinterpret_cast<const char*>(data + foot_off + 1), e - foot_off - 1));
    }
  }
  z->fixed = false;
  if (z->trans.empty() && (!z->footer.valid || !z->footer.has_dst)) {
    z->fixed = true;
    z->fixed_off = z->footer.valid ? z->footer.std_off : utoff[0];
  }
  return true;
}

int add_zone(std::shared_ptr<Zone> z) {
  std::lock_guard<std::mutex> lk(g_zone_mu);
  g_zones.push_back(std::move(z));
  return static_cast<int>(g_zones.size()) - 1;
}

const Zone* get_zone(int id) {
  std::lock_guard<std::mutex> lk(g_zone_mu);
  if (id < 0 || static_cast<size_t>(id) >= g_zones.size()) return nullptr;
  return g_zones[id].get();
}

// ------------------------------------------------------------------ Go time

struct GTime {
  int64_t sec;
  int64_t nsec;
  const Zone* z;
};

struct Fields {
  int64_t year;
  int month, day, hour, minute, second, weekday;
};

inline int64_t offset_of(const GTime& t) { return zone_offset_at(*t.z, t.sec); }

inline Fields fields_of(const GTime& t) {
  const int64_t w = t.sec + offset_of(t);
  const int64_t days = floordiv(w, 86400);
  const int64_t rem = w - days * 86400;
  const Civil c = civil_from_days(days);
  Fields f;
  f.year = c.y;
  f.month = c.m;
  f.day = c.d;
  f.hour = static_cast<int>(rem / 3600);
  f.minute = static_cast<int>((rem / 60) % 60);
  f.second = static_cast<int>(rem % 60);
  f.weekday = static_cast<int>(floormod(days + 4, 7));
  return f;
}

inline GTime add_ns(const GTime& t, int64_t d) {
  const int64_t ns = t.nsec + d;
  return GTime{t.sec + floordiv(ns, kNanos), floormod(ns, kNanos), t.z};
}

// Go time.Date with normalisation and Go's DST resolution.
GTime go_date(int64_t y, int64_t mo, int64_t d, int64_t h, int64_t mi, int64_t s, int64_t ns, const Zone* z) {
  s += floordiv(ns, kNanos);
  ns = floormod(ns, kNanos);
  const int64_t wall = days_from_civil(y, mo, d) * 86400 + h * 3600 + mi * 60 + s;
  if (z->fixed) return GTime{wall - z->fixed_off, ns, z};
  const int64_t off = zone_offset_at(*z, wall - zone_offset_at(*z, wall));
  return GTime{wall - off, ns, z};
}

inline GTime add_date(const GTime& t, int years, int months, int days) {
  const Fields f = fields_of(t);
  return go_date(f.year + years, f.month + months, f.day + days, f.hour, f.minute, f.second, t.nsec, t.z);
}

inline GTime truncate_abs(const GTime& t, int64_t d_ns) {
  // absolute ns since year 1 modulo d (d divides 1 day here, so seconds math suffices)
  const int64_t dsec = d_ns / kNanos;
  const int64_t abs_sec = t.sec + kUnixToAbs;
  const int64_t r = floormod(abs_sec, dsec);
  return GTime{t.sec - r, 0, t.z};
}

// ------------------------------------------------------------------ schedules

struct Spec {
  bool every = false;
  int64_t delay = 0;
  uint64_t second = 0, minute = 0, hour = 0, dom = 0, month = 0, dow = 0;
  int zone = -1;  // -1 = Local (use the time's zone)
};

inline int next_bit(uint64_t mask, int start, int limit) {
  if (start > 63) return -1;
  const uint64_t m = (mask & ~kStarBit) >> start;
  if (m == 0) return -1;
  const int b = __builtin_ctzll(m) + start;
  return b <= limit ? b : -1;
}

inline bool day_matches(const Spec& s, const Fields& f) {
  const bool dm = ((1ULL << f.day) & s.dom) != 0;
  const bool wm = ((1ULL << f.weekday) & s.dow) != 0;
  if ((s.dom & kStarBit) || (s.dow & kStarBit)) return dm && wm;
  return dm || wm;
}

GTime spec_next(const Spec& s, GTime t) {
  if (s.every) return add_ns(t, s.delay - t.nsec);
  const Zone* orig = t.z;
  const Zone* loc = t.z;
  if (s.zone >= 0) {
    loc = get_zone(s.zone);
    t.z = loc;
  }
  t = add_ns(t, kNanos - t.nsec);
  bool added = false;
  const int64_t year_limit = fields_of(t).year + 5;

WRAP:
  {
    Fields f = fields_of(t);
    if (f.year > year_limit) return GTime{kZeroUnix, 0, orig};

    while (((1ULL << f.month) & s.month) == 0) {
      if (!added) {
        added = true;
        t = go_date(f.year, f.month, 1, 0, 0, 0, 0, loc);
      }
      t = add_date(t, 0, 1, 0);
      f = fields_of(t);
      if (f.month == 1) goto WRAP;
    }

    while (!day_matches(s, f)) {
      if (!added) {
        added = true;
        t = go_date(f.year, f.month, f.day, 0, 0, 0, 0, loc);
      }
      t = add_date(t, 0, 0, 1);
      f = fields_of(t);
      if (f.hour != 0) {
        if (f.hour > 12) {
          t = add_ns(t, static_cast<int64_t>(24 - f.hour) * 3600 * kNanos);
        } else {
          t = add_ns(t, -static_cast<int64_t>(f.hour) * 3600 * kNanos);
        }
        f = fields_of(t);
      }
      if (f.day == 1) goto WRAP;
    }

    while (((1ULL << f.hour) & s.hour) == 0) {
      if (!added) {
        added = true;
        t = go_date(f.year, f.month, f.day, f.hour, 0, 0, 0, loc);
        f = fields_of(t);
      }
      const int cur = f.hour;
      const int nb = next_bit(s.hour, cur + 1, 23);
      const int steps = nb >= 0 ? nb - cur : 24 - cur;
      GTime cand = add_ns(t, static_cast<int64_t>(steps) * 3600 * kNanos);
      if (steps > 1 && !zone_constant_between(*t.z, t.sec, cand.sec)) cand = add_ns(t, 3600 * kNanos);
      t = cand;
      f = fields_of(t);
      if (f.hour == 0) goto WRAP;
    }

    while (((1ULL << f.minute) & s.minute) == 0) {
      if (!added) {
        added = true;
        t = truncate_abs(t, 60 * kNanos);
        f = fields_of(t);
      }
      const int cur = f.minute;
      const int nb = next_bit(s.minute, cur + 1, 59);
      const int steps = nb >= 0 ? nb - cur : 60 - cur;
      GTime cand = add_ns(t, static_cast<int64_t>(steps) * 60 * kNanos);
      if (steps > 1 && !zone_constant_between(*t.z, t.sec, cand.sec)) cand = add_ns(t, 60 * kNanos);
      t = cand;
      f = fields_of(t);
      if (f.minute == 0) goto WRAP;
    }

    while (((1ULL << f.second) & s.second) == 0) {
      if (!added) {
        added = true;
        t = truncate_abs(t, kNanos);
        f = fields_of(t);
      }
      const int cur = f.second;
      const int nb = next_bit(s.second, cur + 1, 59);
      const int steps = nb >= 0 ? nb - cur : 60 - cur;
      GTime cand = add_ns(t, static_cast<int64_t>(steps) * kNanos);
      if (steps > 1 && !zone_constant_between(*t.z, t.sec, cand.sec)) cand = add_ns(t, kNanos);
      t = cand;
      f = fields_of(t);
      if (f.second == 0) goto WRAP;
    }
  }
  t.z = orig;
  return t;
}

inline bool is_zero(const GTime& t) { return t.sec == kZeroUnix && t.nsec == 0; }
inline bool after(const GTime& a, const GTime& b) { return a.sec > b.sec || (a.sec == b.sec && a.nsec > b.nsec); }

int popcount_range(uint64_t mask, int lo, int hi) {
  int n = 0;
  for (int i = lo; i <= hi; ++i) n += (mask >> i) & 1;
  return n;
}

// Whole-day tick counting for the missed-run scan.  For a constant-offset zone
// every local day has all 24 hours, so a matching day contributes exactly
// |hours| * |minutes| * |seconds| ticks.  `ok` is false when two consecutive
// matching days are more than four years apart: Next() gives up after five
// calendar years, so such a gap must be walked tick by tick to reproduce the
// zero-time ("unschedulable") result exactly.
struct FullDays {
  int64_t count = 0;
  int64_t last_day = INT64_MIN;
  bool ok = true;
};

int highest_bit(uint64_t mask, int hi) {
  for (int i = hi; i >= 0; --i)
    if ((mask >> i) & 1) return i;
  return -1;
}

FullDays count_full_days(const Spec& s, int64_t d0, int64_t d1, int64_t prev_match) {
  FullDays fd;
  const int64_t per_day = int64_t(popcount_range(s.hour, 0, 23)) * popcount_range(s.minute, 0, 59) *
                          popcount_range(s.second, 0, 59);
  if (per_day == 0) {
    fd.ok = false;
    return fd;
  }
  int64_t prev = prev_match;
  for (int64_t d = d0; d < d1; ++d) {
    const Civil c = civil_from_days(d);
    if (((1ULL << c.m) & s.month) == 0) continue;
    Fields f{};
    f.day = c.d;
    f.weekday = static_cast<int>(floormod(d + 4, 7));
    if (!day_matches(s, f)) continue;
    if (d - prev > 1461) {
      fd.ok = false;
      return fd;
    }
    prev = d;
    fd.count += per_day;
    fd.last_day = d;
  }
  return fd;
}

struct Missed {
  GTime last;
  int64_t count;
  bool unschedulable;
};

// Exact equivalent of the reference loop (cron_controller.go:409-430):
//   for t = Next(earliest); !t.After(now); t = Next(t) { lastMissed = t; count++ }
// with whole days counted in closed form when the zone offset is constant.
Missed missed_runs(const Spec& s, GTime earliest, GTime now) {
  const GTime zero{kZeroUnix, 0, earliest.z};
  Missed r{zero, 0, false};
  GTime t = spec_next(s, earliest);
  const Zone* sz = (!s.every && s.zone >= 0) ? get_zone(s.zone) : earliest.z;
  if (!s.every && !is_zero(t) && sz && now.sec - t.sec > 3 * 86400 && zone_constant_between(*sz, t.sec, now.sec)) {
    const int64_t off = zone_offset_at(*sz, t.sec);
    const int64_t day0 = floordiv(t.sec + off, 86400);
    const int64_t nowday = floordiv(now.sec + off, 86400);
    while (!after(t, now) && floordiv(t.sec + off, 86400) == day0) {
      if (is_zero(t)) {
        r.last = zero;
        r.unschedulable = true;
        return r;
      }
      r.last = t;
      r.count++;
      t = spec_next(s, t);
    }
    if (nowday - 1 > day0 && !is_zero(t) && !after(t, now)) {
      const FullDays fd = count_full_days(s, day0 + 1, nowday, day0);
      if (fd.ok && fd.count > 0) {
        const int h = highest_bit(s.hour, 23), m = highest_bit(s.minute, 59), sec = highest_bit(s.second, 59);
        r.count += fd.count;
        r.last = GTime{fd.last_day * 86400 + h * 3600 + m * 60 + sec - off, 0, earliest.z};
        t = spec_next(s, r.last);
      }
    }
  }
  while (!after(t, now)) {
    if (is_zero(t)) {
      r.last = zero;
      r.unschedulable = true;
      return r;
    }
    r.last = t;
    r.count++;
    t = spec_next(s, t);
  }
  return r;
}

// ------------------------------------------------------------------ parser

struct ParseErr {
  std::string msg;
};

struct Bounds {
  int lo, hi;
  int names;  // 0 none, 1 months, 2 weekdays
};

const Bounds kSeconds{0, 59, 0}, kMinutes{0, 59, 0}, kHours{0, 23, 0}, kDom{1, 31, 0}, kMonths{1, 12, 1},
    kDow{0, 6, 2};

std::string lower(const std::string& s) {
  std::string o = s;
  for (auto& c : o) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return o;
}

bool lookup_name(const std::string& e, int which, int64_t* out) {
  static const char* kMon[] = {"jan", "feb", "mar", "apr", "may", "jun", "jul", "aug", "sep", "oct", "nov", "dec"};
  static const char* kDay[] = {"sun", "mon", "tue", "wed", "thu", "fri", "sat"};
  const std::string l = lower(e);
  if (which == 1) {
    for (int i = 0; i < 12; ++i)
      if (l == kMon[i]) {
        *out = i + 1;
        return true;
      }
  } else if (which == 2) {
    for (int i = 0; i < 7; ++i)
      if (l == kDay[i]) {
        *out = i;
        return true;
      }
  }
  return false;
}

int64_t atoi_go(const std::string& expr) {
  size_t i = 0;
  bool neg = false;
  if (!expr.empty() && (expr[0] == '+' || expr[0] == '-')) {
    neg = expr[0] == '-';
    i = 1;
  }
  if (i >= expr.size()) throw ParseErr{"failed to parse int from " + expr + ": strconv.Atoi: parsing \"" + expr + "\": invalid syntax"};
  __int128 v = 0;
  for (; i < expr.size(); ++i) {
    const char c = expr[i];
    if (c < '0' || c > '9')
      throw ParseErr{"failed to parse int from " + expr + ": strconv.Atoi: parsing \"" + expr + "\": invalid syntax"};
    v = v * 10 + (c - '0');
    if (v > (__int128(1) << 64))
      throw ParseErr{"failed to parse int from " + expr + ": strconv.Atoi: parsing \"" + expr + "\": value out of range"};
  }
  if (neg) v = -v;
  if (v > INT64_MAX || v < INT64_MIN)
    throw ParseErr{"failed to parse int from " + expr + ": strconv.Atoi: parsing \"" + expr + "\": value out of range"};
  return static_cast<int64_t>(v);
}

int64_t must_parse_int(const std::string& expr) {
  const int64_t n = atoi_go(expr);
  if (n < 0) throw ParseErr{"negative number (" + std::to_string(n) + ") not allowed: " + expr};
  return n;
}

int64_t int_or_name(const std::string& e, const Bounds& r) {
  int64_t v;
  if (r.names && lookup_name(e, r.names, &v)) return v;
  return must_parse_int(e);
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  size_t b = 0;
  while (true) {
    const size_t e = s.find(sep, b);
    if (e == std::string::npos) {
      out.push_back(s.substr(b));
      break;
    }
    out.push_back(s.substr(b, e - b));
    b = e + 1;
  }
  return out;
}

uint64_t bits(int64_t lo, int64_t hi, int64_t step) {
  uint64_t o = 0;
  for (int64_t i = lo; i <= hi; i += step) o |= 1ULL << i;
  return o;
}

uint64_t get_range(const std::string& expr, const Bounds& r) {
  const auto rs = split(expr, '/');
  const auto lh = split(rs[0], '-');
  const bool single = lh.size() == 1;
  uint64_t extra = 0;
  int64_t start, end, step;
  if (lh[0] == "*" || lh[0] == "?") {
    start = r.lo;
    end = r.hi;
    extra = kStarBit;
  } else {
    start = int_or_name(lh[0], r);
    if (lh.size() == 1) {
      end = start;
    } else if (lh.size() == 2) {
      end = int_or_name(lh[1], r);
    } else {
      throw ParseErr{"too many hyphens: " + expr};
    }
  }
  if (rs.size() == 1) {
    step = 1;
  } else if (rs.size() == 2) {
    step = must_parse_int(rs[1]);
    if (single) end = r.hi;
    if (step > 1) extra = 0;
  } else {
    throw ParseErr{"too many slashes: " + expr};
  }
  if (start < r.lo)
    throw ParseErr{"beginning of range (" + std::to_string(start) + ") below minimum (" + std::to_string(r.lo) + "): " + expr};
  if (end > r.hi)
    throw ParseErr{"end of range (" + std::to_string(end) + ") above maximum (" + std::to_string(r.hi) + "): " + expr};
  if (start > end)
    throw ParseErr{"beginning of range (" + std::to_string(start) + ") beyond end of range (" + std::to_string(end) + "): " + expr};
  if (step == 0) throw ParseErr{"step of range should be a positive number: " + expr};
  return bits(start, end, step) | extra;
}

uint64_t get_field(const std::string& field, const Bounds& r) {
  uint64_t b = 0;
  for (const auto& e : split(field, ',')) {
    if (e.empty()) continue;
    b |= get_range(e, r);
  }
  return b;
}

uint64_t all_of(const Bounds& r) { return bits(r.lo, r.hi, 1) | kStarBit; }

// Python-side callback that resolves a zone name to a zone id (set by the wrapper).
PyObject* g_zone_resolver = nullptr;

int resolve_zone(const std::string& name) {
  if (name.empty() || name == "UTC") return 0;
  if (name == "Local") return -1;
  if (!g_zone_resolver) throw ParseErr{"provided bad location " + name + ": unknown time zone " + name};
  PyObject* r = PyObject_CallFunction(g_zone_resolver, "s#", name.data(), static_cast<Py_ssize_t>(name.size()));
  if (!r) {
    PyErr_Clear();
    throw ParseErr{"provided bad location " + name + ": unknown time zone " + name};
  }
  const long id = PyLong_AsLong(r);
  Py_DECREF(r);
  if (id < 0 || PyErr_Occurred()) {
    PyErr_Clear();
    throw ParseErr{"provided bad location " + name + ": unknown time zone " + name};
  }
  return static_cast<int>(id);
}

int64_t parse_go_duration(const std::string& s);

Spec parse_spec(std::string spec) {
  if (spec.empty()) throw ParseErr{"empty spec string"};
  int zone = -1;
  if (spec.rfind("TZ=", 0) == 0 || spec.rfind("CRON_TZ=", 0) == 0) {
    const size_t i = spec.find(' ');
    const size_t eq = spec.find('=');
    if (i == std::string::npos)
      throw ParseErr{"provided bad location " + spec.substr(eq + 1) + ": missing schedule after time zone"};
    zone = resolve_zone(spec.substr(eq + 1, i - eq - 1));
    // strings.TrimSpace
    size_t b = i, e = spec.size();
    while (b < e && std::isspace(static_cast<unsigned char>(spec[b]))) ++b;
    while (e > b && std::isspace(static_cast<unsigned char>(spec[e - 1]))) --e;
    spec = spec.substr(b, e - b);
  }
  Spec s;
  s.zone = zone;
  if (!spec.empty() && spec[0] == '@') {
    const uint64_t one_s = 1ULL << kSeconds.lo, one_m = 1ULL << kMinutes.lo, one_h = 1ULL << kHours.lo,
                   one_d = 1ULL << kDom.lo, one_mo = 1ULL << kMonths.lo, one_w = 1ULL << kDow.lo;
    if (spec == "@yearly" || spec == "@annually") {
      s.second = one_s, s.minute = one_m, s.hour = one_h, s.dom = one_d, s.month = one_mo, s.dow = all_of(kDow);
    } else if (spec == "@monthly") {
      s.second = one_s, s.minute = one_m, s.hour = one_h, s.dom = one_d, s.month = all_of(kMonths), s.dow = all_of(kDow);
    } else if (spec == "@weekly") {
      s.second = one_s, s.minute = one_m, s.hour = one_h, s.dom = all_of(kDom), s.month = all_of(kMonths), s.dow = one_w;
    } else if (spec == "@daily" || spec == "@midnight") {
      s.second = one_s, s.minute = one_m, s.hour = one_h, s.dom = all_of(kDom), s.month = all_of(kMonths), s.dow = all_of(kDow);
    } else if (spec == "@hourly") {
      s.second = one_s, s.minute = one_m, s.hour = all_of(kHours), s.dom = all_of(kDom), s.month = all_of(kMonths),
      s.dow = all_of(kDow);
    } else if (spec.rfind("@every ", 0) == 0) {
      int64_t d;
      try {
        d = parse_go_duration(spec.substr(7));
      } catch (const ParseErr& e) {
        throw ParseErr{"failed to parse duration " + spec + ": " + e.msg};
      }
      if (d < kNanos) d = kNanos;
      s.every = true;
      s.delay = d - d % kNanos;
      s.zone = -1;
    } else {
      throw ParseErr{"unrecognized descriptor: " + spec};
    }
    return s;
  }
  // strings.Fields (ASCII whitespace; Unicode spaces are rejected by Python before the call)
  std::vector<std::string> f;
  size_t i = 0;
  while (i < spec.size()) {
    while (i < spec.size() && std::isspace(static_cast<unsigned char>(spec[i]))) ++i;
    if (i >= spec.size()) break;
    size_t j = i;
    while (j < spec.size() && !std::isspace(static_cast<unsigned char>(spec[j]))) ++j;
    f.push_back(spec.substr(i, j - i));
    i = j;
  }
  if (f.size() != 5) {
    std::string joined;
    for (size_t k = 0; k < f.size(); ++k) joined += (k ? " " : "") + f[k];
    throw ParseErr{"expected exactly 5 fields, found " + std::to_string(f.size()) + ": [" + joined + "]"};
  }
  s.second = get_field("0", kSeconds);
  s.minute = get_field(f[0], kMinutes);
  s.hour = get_field(f[1], kHours);
  s.dom = get_field(f[2], kDom);
  s.month = get_field(f[3], kMonths);
  s.dow = get_field(f[4], kDow);
  return s;
}

int64_t parse_go_duration(const std::string& orig) {
  std::string s = orig;
  const std::string bad = "time: invalid duration \"" + orig + "\"";
  if (s.empty()) throw ParseErr{bad};
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    s = s.substr(1);
  }
  if (s == "0") return 0;
  if (s.empty()) throw ParseErr{bad};
  __int128 total = 0;
  size_t p = 0;
  while (p < s.size()) {
    size_t q = p;
    while (q < s.size() && std::isdigit(static_cast<unsigned char>(s[q]))) ++q;
    const std::string whole = s.substr(p, q - p);
    p = q;
    std::string frac;
    if (p < s.size() && s[p] == '.') {
      ++p;
      q = p;
      while (q < s.size() && std::isdigit(static_cast<unsigned char>(s[q]))) ++q;
      frac = s.substr(p, q - p);
      p = q;
    }
    if (whole.empty() && frac.empty()) throw ParseErr{bad};
    q = p;
    while (q < s.size() && s[q] != '.' && !std::isdigit(static_cast<unsigned char>(s[q]))) ++q;
    if (q == p) throw ParseErr{"time: missing unit in duration \"" + orig + "\""};
    const std::string unit = s.substr(p, q - p);
    p = q;
    int64_t scale;
    if (unit == "ns") scale = 1;
    else if (unit == "us" || unit == "\xc2\xb5s" || unit == "\xce\xbcs") scale = 1000;
    else if (unit == "ms") scale = 1000000;
    else if (unit == "s") scale = kNanos;
    else if (unit == "m") scale = 60 * kNanos;
    else if (unit == "h") scale = 3600 * kNanos;
    else throw ParseErr{"time: unknown unit \"" + unit + "\" in duration \"" + orig + "\""};
    __int128 v = 0;
    for (char c : whole) {
      v = v * 10 + (c - '0');
      if (v > (__int128(INT64_MAX))) throw ParseErr{bad};
    }
    v *= scale;
    if (v > (__int128(INT64_MAX))) throw ParseErr{bad};
    if (!frac.empty()) {
      double fv = 0, sc = 1;
      for (char c : frac) {
        fv = fv * 10 + (c - '0');
        sc *= 10;
      }
      v += static_cast<int64_t>(fv * (static_cast<double>(scale) / sc));
    }
    total += v;
    if (total > (__int128(INT64_MAX) + (neg ? 1 : 0))) throw ParseErr{bad};
  }
  return static_cast<int64_t>(neg ? -total : total);
}

// ------------------------------------------------------------------ Python bindings

struct PySchedule {
  PyObject_HEAD Spec spec;
};

extern PyTypeObject PyScheduleType;

const Zone* zone_arg(long id) {
  const Zone* z = get_zone(static_cast<int>(id));
  if (!z) PyErr_Format(PyExc_ValueError, "unknown zone id %ld", id);
  return z;
}

PyObject* sched_next(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "next(sec, nsec, zone)");
    return nullptr;
  }
  const long long sec = PyLong_AsLongLong(args[0]);
  const long long nsec = PyLong_AsLongLong(args[1]);
  const long zid = PyLong_AsLong(args[2]);
  if (PyErr_Occurred()) return nullptr;
  const Zone* z = zone_arg(zid);
  if (!z) return nullptr;
  const GTime r = spec_next(reinterpret_cast<PySchedule*>(self)->spec, GTime{sec, nsec, z});
  return Py_BuildValue("(LL)", static_cast<long long>(r.sec), static_cast<long long>(r.nsec));
}

PyObject* sched_missed(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 5) {
    PyErr_SetString(PyExc_TypeError, "missed(e_sec, e_nsec, n_sec, n_nsec, zone)");
    return nullptr;
  }
  const long long es = PyLong_AsLongLong(args[0]), en = PyLong_AsLongLong(args[1]);
  const long long ns = PyLong_AsLongLong(args[2]), nn = PyLong_AsLongLong(args[3]);
  const long zid = PyLong_AsLong(args[4]);
  if (PyErr_Occurred()) return nullptr;
  const Zone* z = zone_arg(zid);
  if (!z) return nullptr;
  Missed m;
  Py_BEGIN_ALLOW_THREADS m = missed_runs(reinterpret_cast<PySchedule*>(self)->spec, GTime{es, en, z}, GTime{ns, nn, z});
  Py_END_ALLOW_THREADS return Py_BuildValue("(LLLO)", static_cast<long long>(m.last.sec),
                                            static_cast<long long>(m.last.nsec), static_cast<long long>(m.count),
                                            m.unschedulable ? Py_True : Py_False);
}

PyObject* sched_masks(PyObject* self, PyObject*) {
  const Spec& s = reinterpret_cast<PySchedule*>(self)->spec;
  return Py_BuildValue("(KKKKKKi)", static_cast<unsigned long long>(s.second), static_cast<unsigned long long>(s.minute),
                       static_cast<unsigned long long>(s.hour), static_cast<unsigned long long>(s.dom),
                       static_cast<unsigned long long>(s.month), static_cast<unsigned long long>(s.dow), s.zone);
}

PyObject* sched_get_every(PyObject* self, void*) {
  return PyBool_FromLong(reinterpret_cast<PySchedule*>(self)->spec.every);
}
PyObject* sched_get_delay(PyObject* self, void*) {
  return PyLong_FromLongLong(reinterpret_cast<PySchedule*>(self)->spec.delay);
}

PyMethodDef sched_methods[] = {
    {"next", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(sched_next)), METH_FASTCALL,
     "next(sec, nsec, zone) -> (sec, nsec)"},
    {"missed", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(sched_missed)), METH_FASTCALL,
     "missed(e_sec, e_nsec, n_sec, n_nsec, zone) -> (last_sec, last_nsec, count, unschedulable)"},
    {"masks", sched_masks, METH_NOARGS, "field masks + zone id"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef sched_getset[] = {{"is_every", sched_get_every, nullptr, nullptr, nullptr},
                              {"delay", sched_get_delay, nullptr, nullptr, nullptr},
                              {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject PyScheduleType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyObject* py_parse(PyObject*, PyObject* arg) {
  Py_ssize_t n;
  const char* p = PyUnicode_AsUTF8AndSize(arg, &n);
  if (!p) return nullptr;
  Spec s;
  try {
    s = parse_spec(std::string(p, n));
  } catch (const ParseErr& e) {
    PyErr_SetString(PyExc_ValueError, e.msg.c_str());
    return nullptr;
  }
  PySchedule* o = PyObject_New(PySchedule, &PyScheduleType);
  if (!o) return nullptr;
  o->spec = s;
  return reinterpret_cast<PyObject*>(o);
}

PyObject* py_register_zone(PyObject*, PyObject* args) {
  const char* name;
  Py_buffer buf;
  if (!PyArg_ParseTuple(args, "sy*", &name, &buf)) return nullptr;
  auto z = std::make_shared<Zone>();
  z->name = name;
  std::string err;
  const bool ok = parse_tzif(static_cast<const uint8_t*>(buf.buf), static_cast<size_t>(buf.len), z.get(), &err);
  PyBuffer_Release(&buf);
  if (!ok) {
    PyErr_Format(PyExc_ValueError, "bad TZif data for %s: %s", name, err.c_str());
    return nullptr;
  }
  return PyLong_FromLong(add_zone(z));
}

PyObject* py_register_fixed(PyObject*, PyObject* args) {
  const char* name;
  long long off;
  if (!PyArg_ParseTuple(args, "sL", &name, &off)) return nullptr;
  auto z = std::make_shared<Zone>();
  z->name = name;
  z->fixed = true;
  z->fixed_off = off;
  return PyLong_FromLong(add_zone(z));
}

PyObject* py_zone_offset(PyObject*, PyObject* args) {
  long id;
  long long unix;
  if (!PyArg_ParseTuple(args, "lL", &id, &unix)) return nullptr;
  const Zone* z = zone_arg(id);
  if (!z) return nullptr;
  return PyLong_FromLongLong(zone_offset_at(*z, unix));
}

PyObject* py_set_zone_resolver(PyObject*, PyObject* fn) {
  Py_XINCREF(fn);
  Py_XDECREF(g_zone_resolver);
  g_zone_resolver = fn == Py_None ? nullptr : fn;
  if (fn == Py_None) Py_DECREF(fn);
  Py_RETURN_NONE;
}

PyObject* py_go_date(PyObject*, PyObject* args) {
  long long y, mo, d, h, mi, s, ns;
  long zid;
  if (!PyArg_ParseTuple(args, "LLLLLLLl", &y, &mo, &d, &h, &mi, &s, &ns, &zid)) return nullptr;
  const Zone* z = zone_arg(zid);
  if (!z) return nullptr;
  const GTime t = go_date(y, mo, d, h, mi, s, ns, z);
  return Py_BuildValue("(LL)", static_cast<long long>(t.sec), static_cast<long long>(t.nsec));
}

// bulk_next(schedules, secs, nsecs, zone) -> list of (sec, nsec)
PyObject* py_bulk_next(PyObject*, PyObject* args) {
  PyObject *scheds, *secs, *nsecs;
  long zid;
  if (!PyArg_ParseTuple(args, "OOOl", &scheds, &secs, &nsecs, &zid)) return nullptr;
  const Zone* z = zone_arg(zid);
  if (!z) return nullptr;
  PyObject* fs = PySequence_Fast(scheds, "schedules must be a sequence");
  if (!fs) return nullptr;
  PyObject* fsec = PySequence_Fast(secs, "secs must be a sequence");
  PyObject* fnsec = fsec ? PySequence_Fast(nsecs, "nsecs must be a sequence") : nullptr;
  if (!fsec || !fnsec) {
    Py_DECREF(fs);
    Py_XDECREF(fsec);
    return nullptr;
  }
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(fs);
  if (PySequence_Fast_GET_SIZE(fsec) != n || PySequence_Fast_GET_SIZE(fnsec) != n) {
    Py_DECREF(fs);
    Py_DECREF(fsec);
    Py_DECREF(fnsec);
    PyErr_SetString(PyExc_ValueError, "length mismatch");
    return nullptr;
  }
  std::vector<Spec> sp(n);
  std::vector<GTime> tt(n);
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyObject* o = PySequence_Fast_GET_ITEM(fs, i);
    if (!PyObject_TypeCheck(o, &PyScheduleType)) {
      Py_DECREF(fs);
      Py_DECREF(fsec);
      Py_DECREF(fnsec);
      PyErr_SetString(PyExc_TypeError, "expected Schedule");
      return nullptr;
    }
    sp[i] = reinterpret_cast<PySchedule*>(o)->spec;
    tt[i] = GTime{PyLong_AsLongLong(PySequence_Fast_GET_ITEM(fsec, i)),
                  PyLong_AsLongLong(PySequence_Fast_GET_ITEM(fnsec, i)), z};
  }
  Py_DECREF(fs);
  Py_DECREF(fsec);
  Py_DECREF(fnsec);
  if (PyErr_Occurred()) return nullptr;
  Py_BEGIN_ALLOW_THREADS for (Py_ssize_t i = 0; i < n; ++i) tt[i] = spec_next(sp[i], tt[i]);
  Py_END_ALLOW_THREADS PyObject* out = PyList_New(n);
  if (!out) return nullptr;
  for (Py_ssize_t i = 0; i < n; ++i) {
    PyList_SET_ITEM(out, i, Py_BuildValue("(LL)", static_cast<long long>(tt[i].sec), static_cast<long long>(tt[i].nsec)));
  }
  return out;
}

PyObject* py_parse_duration(PyObject*, PyObject* arg) {
  Py_ssize_t n;
  const char* p = PyUnicode_AsUTF8AndSize(arg, &n);
  if (!p) return nullptr;
  try {
    return PyLong_FromLongLong(parse_go_duration(std::string(p, n)));
  } catch (const ParseErr& e) {
    PyErr_SetString(PyExc_ValueError, e.msg.c_str());
    return nullptr;
  }
}

// ------------------------------------------------------------------ RFC 3339 timestamps
//
// metav1.Time is written as "YYYY-MM-DDTHH:MM:SSZ"; every child event and status write carries a
// few new ones, so these replace the Python arithmetic of utils/gotime.py for that exact shape.
// Anything else returns None and the Python code decides (same results, tests/test_gotime.py).

inline int digits(const Py_UCS1* p, int n) {
  int v = 0;
  for (int i = 0; i < n; ++i) {
    if (p[i] < '0' || p[i] > '9') return -1;
    v = v * 10 + (p[i] - '0');
  }
  return v;
}

// rfc3339_z(s) -> unix seconds | None
PyObject* py_rfc3339_z(PyObject*, PyObject* arg) {
  if (!PyUnicode_Check(arg)) {
    PyErr_SetString(PyExc_TypeError, "rfc3339_z expects str");
    return nullptr;
  }
  if (PyUnicode_READY(arg) < 0) return nullptr;
  if (PyUnicode_GET_LENGTH(arg) != 20 || PyUnicode_KIND(arg) != PyUnicode_1BYTE_KIND) Py_RETURN_NONE;
  const Py_UCS1* s = PyUnicode_1BYTE_DATA(arg);
  if (s[4] != '-' || s[7] != '-' || s[10] != 'T' || s[13] != ':' || s[16] != ':' || s[19] != 'Z') Py_RETURN_NONE;
  const int y = digits(s, 4), mo = digits(s + 5, 2), d = digits(s + 8, 2);
  const int hh = digits(s + 11, 2), mi = digits(s + 14, 2), ss = digits(s + 17, 2);
  if (y < 0 || mo < 1 || mo > 12 || d < 1 || d > 31 || hh < 0 || hh > 23 || mi < 0 || mi > 59 || ss < 0 || ss > 59)
    Py_RETURN_NONE;
  return PyLong_FromLongLong(days_from_civil(y, mo, d) * 86400 + hh * 3600 + mi * 60 + ss);
}

// format_rfc3339(wall, nsec, offset) -> str | None: Go's RFC 3339 of the wall-clock second `wall`
// (unix seconds + offset), fractional nanoseconds without trailing zeros when nsec != 0, and "Z"
// or "+hh:mm" for the offset; None outside years 0..9999
PyObject* py_format_rfc3339(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "format_rfc3339(wall, nsec, offset)");
    return nullptr;
  }
  const long long wall = PyLong_AsLongLong(args[0]);
  const long long nsec = PyLong_AsLongLong(args[1]);
  const long long off = PyLong_AsLongLong(args[2]);
  if (PyErr_Occurred()) return nullptr;
  if (nsec < 0 || nsec >= 1000000000LL || off <= -360000 || off >= 360000) Py_RETURN_NONE;
  const int64_t days = floordiv(wall, 86400);
  const int64_t rem = wall - days * 86400;
  const Civil c = civil_from_days(days);
  if (c.y < 0 || c.y > 9999) Py_RETURN_NONE;
  char buf[48];
  int n = std::snprintf(buf, sizeof buf, "%04d-%02d-%02dT%02d:%02d:%02d", static_cast<int>(c.y), c.m, c.d,
                        static_cast<int>(rem / 3600), static_cast<int>((rem / 60) % 60), static_cast<int>(rem % 60));
  if (nsec) {
    char frac[16];
    std::snprintf(frac, sizeof frac, "%09lld", nsec);
    int k = 9;
    while (k > 0 && frac[k - 1] == '0') --k;
    buf[n++] = '.';
    std::memcpy(buf + n, frac, static_cast<size_t>(k));
    n += k;
  }
  if (off == 0) {
    buf[n++] = 'Z';
  } else {
    const long long a = off < 0 ? -off : off;
    n += std::snprintf(buf + n, sizeof buf - static_cast<size_t>(n), "%c%02lld:%02lld", off > 0 ? '+' : '-',
                       a / 3600, (a / 60) % 60);
  }
  return PyUnicode_FromStringAndSize(buf, n);
}

PyMethodDef module_methods[] = {
    {"parse", py_parse, METH_O, "parse(spec) -> Schedule"},
    {"rfc3339_z", py_rfc3339_z, METH_O, "rfc3339_z(s) -> unix seconds of 'YYYY-MM-DDTHH:MM:SSZ', else None"},
    {"format_rfc3339", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(py_format_rfc3339)),
     METH_FASTCALL, "format_rfc3339(wall, nsec, offset) -> str | None"},
    {"register_zone", py_register_zone, METH_VARARGS, "register_zone(name, tzif_bytes) -> id"},
    {"register_fixed_zone", py_register_fixed, METH_VARARGS, "register_fixed_zone(name, offset) -> id"},
    {"zone_offset", py_zone_offset, METH_VARARGS, "zone_offset(id, unix) -> seconds east of UTC"},
    {"set_zone_resolver", py_set_zone_resolver, METH_O, "set_zone_resolver(callable(name)->id)"},
    {"go_date", py_go_date, METH_VARARGS, "go_date(y, mo, d, h, mi, s, ns, zone) -> (sec, nsec)"},
    {"bulk_next", py_bulk_next, METH_VARARGS, "bulk_next(schedules, secs, nsecs, zone) -> [(sec, nsec)]"},
    {"parse_duration", py_parse_duration, METH_O, "Go time.ParseDuration -> ns"},
    {nullptr, nullptr, 0, nullptr}};

PyModuleDef module_def = {PyModuleDef_HEAD_INIT, "_cron_engine", "Native cron next-fire engine", -1, module_methods,
                          nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__cron_engine(void) {
  PyScheduleType.tp_name = "_cron_engine.Schedule";
  PyScheduleType.tp_basicsize = sizeof(PySchedule);
  PyScheduleType.tp_flags = Py_TPFLAGS_DEFAULT;
  PyScheduleType.tp_doc = "Parsed cron schedule";
  PyScheduleType.tp_methods = sched_methods;
  PyScheduleType.tp_getset = sched_getset;
  if (PyType_Ready(&PyScheduleType) < 0) return nullptr;
  {
    auto utc = std::make_shared<Zone>();
    utc->name = "UTC";
    std::lock_guard<std::mutex> lk(g_zone_mu);
    if (g_zones.empty()) g_zones.push_back(utc);  // zone id 0 = UTC
  }
  PyObject* m = PyModule_Create(&module_def);
  if (!m) return nullptr;
  Py_INCREF(&PyScheduleType);
  PyModule_AddObject(m, "Schedule", reinterpret_cast<PyObject*>(&PyScheduleType));
  PyModule_AddIntConstant(m, "ZERO_UNIX", static_cast<long>(kZeroUnix));
  return m;
}
