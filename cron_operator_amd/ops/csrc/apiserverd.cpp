// `_apiserverd`: the fake Kubernetes apiserver's hot path in C++ -- store, admission, watch
// fan-out and the HTTP/1.1 (+TLS) front end, on one epoll thread that never takes the GIL.
//
// Why: in the 1000-Cron benchmark the Python fake apiserver (apiserver/server.py + http.py) sat
// 86-94% busy on one core, so the headline measured the fixture, not the operator (round-5
// verdict #1).  This is the same contract -- the REST paths, merge-patch and /status semantics,
// resourceVersions, label-selected LIST/WATCH with resume and synthetic ADDED events, CRD
// structural-schema prune/default/validate, AlreadyExists/NotFound/Conflict Status bodies,
// finalizers, the per-verb latency model -- served natively.  Anything it does not serve
// (the /debug/fake test controls, server-side Table printing, JSON patch, authn/RBAC, ownerRef
// GC) goes to a Python fallback, which reaches the store again through `Server.request`.
// tests/test_apiserverd.py runs one request stream against both implementations and compares.
//
// Threads: the server thread owns everything.  Python entry points release the GIL, then take
// the server's (recursive) lock; the server thread takes the GIL only to call the fallback, and
// never while another thread could hold the lock and wait for the GIL (they released it).
// APISERVERD_STANDALONE compiles the server without CPython (no fallback, no module), for a
// C++-only harness (a gprof build); the tree builds the module.  The sanitizer run
// (scripts/sanitize.py) builds the module with ASan/UBSan and drives it from Python; the
// in-process stack sampler (profile_start/profile_stop) is what the boxes use.
#ifndef APISERVERD_STANDALONE
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#endif

#include <arpa/inet.h>
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <malloc.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <queue>
#include <random>
#include <set>
#include <string>
#include <string_view>
#include <thread>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <x86intrin.h>

#include "jdom.h"

using jdom::Member;
using jdom::Node;
using jdom::Ref;
using jdom::T;

namespace {

// a node's string (pooled) as a std::string, for messages and map keys
inline std::string S(std::string_view v) { return std::string(v); }

// ====================================================================== errors

struct ApiErr {
  int code = 0;
  std::string reason, message;
  Ref details;  // object or null
};

ApiErr mkerr(int code, const std::string& reason, const std::string& msg) {
  ApiErr e;
  e.code = code;
  e.reason = reason;
  e.message = msg;
  return e;
}

std::string qualified(const std::string& resource, const std::string& group) {
  return group.empty() ? resource : resource + "." + group;
}

Ref name_details(const std::string& name, const std::string& group, const std::string& kind) {
  Ref d = jdom::mk_obj();
  d->o.emplace_back("name", jdom::mk_str(name));
  d->o.emplace_back("group", jdom::mk_str(group));
  d->o.emplace_back("kind", jdom::mk_str(kind));
  return d;
}

ApiErr not_found(const std::string& res, const std::string& group, const std::string& name) {
  ApiErr e = mkerr(404, "NotFound", qualified(res, group) + " \"" + name + "\" not found");
  e.details = name_details(name, group, res);
  return e;
}
ApiErr already_exists(const std::string& res, const std::string& group, const std::string& name) {
  ApiErr e = mkerr(409, "AlreadyExists", qualified(res, group) + " \"" + name + "\" already exists");
  e.details = name_details(name, group, res);
  return e;
}
ApiErr conflict(const std::string& res, const std::string& group, const std::string& name, const std::string& why) {
  ApiErr e = mkerr(409, "Conflict", "Operation cannot be fulfilled on " + qualified(res, group) + " \"" + name +
                                        "\": " + why);
  e.details = name_details(name, group, res);
  return e;
}
ApiErr bad_request(const std::string& m) { return mkerr(400, "BadRequest", m); }
const char* kModified = "the object has been modified; please apply your changes to the latest version and try again";

std::string status_body(const ApiErr& e) {
  Ref st = jdom::mk_obj();
  st->o.emplace_back("kind", jdom::mk_str("Status"));
  st->o.emplace_back("apiVersion", jdom::mk_str("v1"));
  st->o.emplace_back("metadata", jdom::mk_obj());
  st->o.emplace_back("status", jdom::mk_str("Failure"));
  st->o.emplace_back("message", jdom::mk_str(e.message));
  st->o.emplace_back("reason", jdom::mk_str(e.reason));
  st->o.emplace_back("code", jdom::mk_num(e.code));
  if (e.details && e.details->is_obj() && !e.details->o.empty()) st->o.emplace_back("details", e.details);
  return jdom::dump(st.get(), 0);
}

// ====================================================================== small helpers

std::string rfc3339(long long now_ns) {
  time_t sec = static_cast<time_t>(now_ns / 1000000000LL);
  if (now_ns < 0 && now_ns % 1000000000LL) --sec;
  // the clock moves in whole seconds between writes: one formatting per second
  static time_t last = -1;
  static std::string last_s;
  if (sec == last) return last_s;
  struct tm tm;
  gmtime_r(&sec, &tm);
  char buf[32];
  strftime(buf, sizeof buf, "%Y-%m-%dT%H:%M:%SZ", &tm);
  last = sec;
  last_s = buf;
  return last_s;
}

bool is_digit(char c) { return c >= '0' && c <= '9'; }

// ^\d{4}-\d{2}-\d{2}[Tt]\d{2}:\d{2}:\d{2}(\.\d+)?([Zz]|[+-]\d{2}:\d{2})$
bool is_date_time(std::string_view s) {
  const char* p = s.data();
  const char* e = p + s.size();
  auto digits = [&](int n) {
    for (int i = 0; i < n; ++i, ++p)
      if (p >= e || !is_digit(*p)) return false;
    return true;
  };
  auto lit = [&](char c) {
    if (p >= e || *p != c) return false;
    ++p;
    return true;
  };
  if (!digits(4) || !lit('-') || !digits(2) || !lit('-') || !digits(2)) return false;
  if (p >= e || (*p != 'T' && *p != 't')) return false;
  ++p;
  if (!digits(2) || !lit(':') || !digits(2) || !lit(':') || !digits(2)) return false;
  if (p < e && *p == '.') {
    ++p;
    if (p >= e || !is_digit(*p)) return false;
    while (p < e && is_digit(*p)) ++p;
  }
  if (p < e && (*p == 'Z' || *p == 'z')) return p + 1 == e;
  if (p < e && (*p == '+' || *p == '-')) {
    ++p;
    return digits(2) && lit(':') && digits(2) && p == e;
  }
  return false;
}

std::string go_type_name(const Node* v) {
  switch (v->t) {
    case T::True:
    case T::False: return "boolean";
    case T::Num:
      return (v->s.find_first_of(".eE") == std::string::npos) ? "integer" : "number";
    case T::Str: return "string";
    case T::Arr: return "array";
    case T::Obj: return "object";
    default: return "null";
  }
}

bool num_is_integral(const Node* v) {
  if (v->s.find_first_of(".eE") == std::string::npos) return true;
  const double d = std::strtod(v->s.c_str(), nullptr);
  return std::isfinite(d) && std::floor(d) == d;
}

std::string uuid4(std::mt19937_64& rng) {
  uint64_t a = rng(), b = rng();
  a = (a & 0xFFFFFFFFFFFF0FFFULL) | 0x0000000000004000ULL;
  b = (b & 0x3FFFFFFFFFFFFFFFULL) | 0x8000000000000000ULL;
  char buf[40];
  snprintf(buf, sizeof buf, "%08x-%04x-%04x-%04x-%012llx", static_cast<unsigned>(a >> 32),
           static_cast<unsigned>((a >> 16) & 0xFFFF), static_cast<unsigned>(a & 0xFFFF),
           static_cast<unsigned>(b >> 48), static_cast<unsigned long long>(b & 0xFFFFFFFFFFFFULL));
  return buf;
}

int hexval(char h) {
  if (h >= '0' && h <= '9') return h - '0';
  if (h >= 'a' && h <= 'f') return h - 'a' + 10;
  if (h >= 'A' && h <= 'F') return h - 'A' + 10;
  return -1;
}

// urllib.parse.unquote (plus=false) / unquote_plus (plus=true); a malformed escape stays as is
std::string url_decode(const std::string& s, bool plus) {
  std::string out;
  out.reserve(s.size());
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (c == '%' && i + 2 < s.size()) {
      const int h1 = hexval(s[i + 1]), h2 = hexval(s[i + 2]);
      if (h1 >= 0 && h2 >= 0) {
        out.push_back(static_cast<char>(h1 * 16 + h2));
        i += 2;
        continue;
      }
    }
    out.push_back(c == '+' && plus ? ' ' : c);
  }
  return out;
}

// parse_qsl(keep_blank_values=True), first value per key
void parse_query(const std::string& qs, std::vector<std::pair<std::string, std::string>>* out) {
  size_t i = 0;
  while (i <= qs.size()) {
    size_t amp = qs.find('&', i);
    if (amp == std::string::npos) amp = qs.size();
    const std::string kv = qs.substr(i, amp - i);
    if (!kv.empty()) {
      const size_t eq = kv.find('=');
      std::string k = url_decode(kv.substr(0, eq), true);
      std::string v = eq == std::string::npos ? std::string() : url_decode(kv.substr(eq + 1), true);
      bool seen = false;
      for (auto& e : *out)
        if (e.first == k) seen = true;
      if (!seen) out->emplace_back(std::move(k), std::move(v));
    }
    i = amp + 1;
  }
}

const char b64url_chars[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789-_";

std::string b64url_encode(const std::string& in) {
  std::string out;
  size_t i = 0;
  while (i + 2 < in.size()) {
    const unsigned v = (static_cast<unsigned char>(in[i]) << 16) | (static_cast<unsigned char>(in[i + 1]) << 8) |
                       static_cast<unsigned char>(in[i + 2]);
    out.push_back(b64url_chars[(v >> 18) & 63]);
    out.push_back(b64url_chars[(v >> 12) & 63]);
    out.push_back(b64url_chars[(v >> 6) & 63]);
    out.push_back(b64url_chars[v & 63]);
    i += 3;
  }
  if (i < in.size()) {
    unsigned v = static_cast<unsigned char>(in[i]) << 16;
    if (i + 1 < in.size()) v |= static_cast<unsigned char>(in[i + 1]) << 8;
    out.push_back(b64url_chars[(v >> 18) & 63]);
    out.push_back(b64url_chars[(v >> 12) & 63]);
    out.push_back(i + 1 < in.size() ? b64url_chars[(v >> 6) & 63] : '=');
    out.push_back('=');
  }
  return out;
}

bool b64url_decode(const std::string& in, std::string* out) {
  unsigned val = 0;  // only the low 14 bits are ever pending: masked, it never overflows
  int bits = -8;
  for (char c : in) {
    if (c == '=') break;
    const char* p = std::strchr(b64url_chars, c);
    if (!p || !*p) return false;
    val = ((val << 6) | static_cast<unsigned>(p - b64url_chars)) & 0xFFFFFFu;
    bits += 6;
    if (bits >= 0) {
      out->push_back(static_cast<char>((val >> bits) & 0xFF));
      bits -= 8;
    }
  }
  return true;
}

// ====================================================================== selectors

struct LabelReq {
  std::string key;
  int op = 0;  // 0 =, 1 !=, 2 in, 3 notin, 4 exists, 5 !exists
  std::vector<std::string> vals;
};

struct FieldReq {
  std::vector<std::string> path;
  bool neq = false;
  std::string val;
};

struct Selector {
  std::vector<LabelReq> labels;
  std::vector<FieldReq> fields;
  bool pinned = false;  // the first `key=value` requirement: every match carries it
  std::string pin_key, pin_val;
  bool labels_only = true;

  static bool tok_char(char c) { return !(c == ' ' || c == '\t' || c == '!' || c == '=' || c == '(' || c == ')' || c == ','); }

  static bool tokens(const std::string& s, std::vector<std::string>* out) {
    size_t i = 0;
    while (i < s.size()) {
      while (i < s.size() && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
      if (i >= s.size()) break;
      if (s.compare(i, 2, "!=") == 0 || s.compare(i, 2, "==") == 0) {
        out->push_back(s.substr(i, 2));
        i += 2;
      } else if (s[i] == '=' || s[i] == '(' || s[i] == ')' || s[i] == ',' || s[i] == '!') {
        out->push_back(s.substr(i, 1));
        ++i;
      } else {
        const size_t b = i;
        while (i < s.size() && tok_char(s[i]) && s[i] != '\n' && s[i] != '\r') ++i;
        if (i == b) return false;
        out->push_back(s.substr(b, i - b));
      }
    }
    return true;
  }

  bool parse_labels(const std::string& s, std::string* err) {
    std::vector<std::string> t;
    if (!tokens(s, &t)) {
      *err = "unable to parse requirement: '" + s + "'";
      return false;
    }
    size_t i = 0;
    while (i < t.size()) {
      LabelReq r;
      if (t[i] == "!") {
        if (i + 1 >= t.size()) {
          *err = "missing key after '!'";
          return false;
        }
        r.key = t[i + 1];
        r.op = 5;
        i += 2;
      } else {
        r.key = t[i++];
        if (i >= t.size() || t[i] == ",") {
          r.op = 4;
        } else if (t[i] == "=" || t[i] == "==" || t[i] == "!=") {
          r.op = t[i] == "!=" ? 1 : 0;
          if (i + 1 >= t.size() || t[i + 1] == ",") {
            r.vals.push_back("");
            i += 1;
          } else {
            r.vals.push_back(t[i + 1]);
            i += 2;
          }
        } else if (t[i] == "in" || t[i] == "notin") {
          r.op = t[i] == "in" ? 2 : 3;
          ++i;
          if (i >= t.size() || t[i] != "(") {
            *err = "expected '(' after " + std::string(r.op == 2 ? "in" : "notin");
            return false;
          }
          ++i;
          while (i < t.size() && t[i] != ")") {
            if (t[i] != ",") r.vals.push_back(t[i]);
            ++i;
          }
          if (i >= t.size()) {
            *err = "unterminated value list";
            return false;
          }
          ++i;
        } else {
          *err = "unexpected token '" + t[i] + "' in selector '" + s + "'";
          return false;
        }
      }
      labels.push_back(std::move(r));
      if (i < t.size()) {
        if (t[i] != ",") {
          *err = "expected ',' in selector '" + s + "'";
          return false;
        }
        ++i;
      }
    }
    for (const auto& r : labels)
      if (r.op == 0) {
        pinned = true;
        pin_key = r.key;
        pin_val = r.vals[0];
        break;
      }
    return true;
  }

  static std::string strip(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
    while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
    return s.substr(b, e - b);
  }

  bool parse_fields(const std::string& s, std::string* err) {
    size_t start = 0;
    while (start <= s.size()) {
      size_t comma = s.find(',', start);
      if (comma == std::string::npos) comma = s.size();
      const std::string part = strip(s.substr(start, comma - start));
      start = comma + 1;
      if (part.empty()) {
        if (comma >= s.size()) break;
        continue;
      }
      FieldReq f;
      size_t pos;
      std::string k, v;
      if ((pos = part.find("!=")) != std::string::npos) {
        k = part.substr(0, pos);
        v = part.substr(pos + 2);
        f.neq = true;
      } else if ((pos = part.find("==")) != std::string::npos) {
        k = part.substr(0, pos);
        v = part.substr(pos + 2);
      } else if ((pos = part.find('=')) != std::string::npos) {
        k = part.substr(0, pos);
        v = part.substr(pos + 1);
      } else {
        *err = "invalid field selector: '" + part + "'";
        return false;
      }
      k = strip(k);
      f.val = strip(v);
      size_t b = 0;
      while (true) {
        const size_t dot = k.find('.', b);
        f.path.push_back(k.substr(b, dot == std::string::npos ? std::string::npos : dot - b));
        if (dot == std::string::npos) break;
        b = dot + 1;
      }
      fields.push_back(std::move(f));
      labels_only = false;
      if (comma >= s.size()) break;
    }
    return true;
  }

  static const jdom::jstr* label(const Node* labels, std::string_view k) {
    if (!labels) return nullptr;
    const Ref* r = labels->get(k);
    if (!r) return nullptr;
    return (*r)->t == T::Str ? &(*r)->s : nullptr;
  }
  static bool in(const std::vector<std::string>& vals, std::string_view v) {
    for (const auto& x : vals)
      if (x == v) return true;
    return false;
  }

  static std::string field_value(const Node* obj, const std::vector<std::string>& path) {
    const Node* cur = obj;
    for (const auto& part : path) {
      if (!cur || !cur->is_obj()) return "\x01";  // None: matches nothing but !=
      const Ref* r = cur->get(part);
      cur = r ? r->get() : nullptr;
    }
    if (!cur || cur->t == T::Null) return "";
    switch (cur->t) {
      case T::Str: return S(cur->s);
      case T::Num: return S(cur->s);
      case T::True: return "True";
      case T::False: return "False";
      default: return jdom::dump(const_cast<Node*>(cur), 0);
    }
  }

  bool empty() const { return labels.empty() && fields.empty(); }

  bool match(const Node* obj) const {
    if (!labels.empty()) {
      const Node* meta = obj->getn("metadata");
      const Node* lb = (meta && meta->is_obj()) ? meta->getn("labels") : nullptr;
      if (lb && !lb->is_obj()) lb = nullptr;
      for (const auto& r : labels) {
        const jdom::jstr* v = label(lb, r.key);
        switch (r.op) {
          case 0:
            if (!v || std::string_view(*v) != r.vals[0]) return false;
            break;
          case 1:
            if (v && std::string_view(*v) == r.vals[0]) return false;
            break;
          case 2:
            if (!v || !in(r.vals, *v)) return false;
            break;
          case 3:
            if (v && in(r.vals, *v)) return false;
            break;
          case 4:
            if (!v) {
              // a non-string label value still "exists"
              if (!(lb && lb->get(r.key))) return false;
            }
            break;
          case 5:
            if (v || (lb && lb->get(r.key))) return false;
            break;
        }
      }
    }
    for (const auto& f : fields) {
      const std::string got = field_value(obj, f.path);
      if (!f.neq && got != f.val) return false;
      if (f.neq && got == f.val) return false;
    }
    return true;
  }
};

// ====================================================================== schema admission

struct Schema {
  std::string type;
  enum class Kind : uint8_t { Any, Object, Array, String, Integer, Number, Boolean } kind = Kind::Any;  // of `type`
  bool nullable = false, preserve = false, date_time = false;
  bool has_enum = false;
  jdom::RefVec enumv;
  bool has_min = false, has_max = false;
  double min = 0, max = 0;
  Ref min_lex, max_lex;
  bool has_props = false;
  std::vector<std::pair<std::string, std::unique_ptr<Schema>>> props;
  std::vector<std::pair<std::string, Ref>> defaults;
  std::vector<std::string> required;
  std::unique_ptr<Schema> addl;
  bool addl_true = false;
  std::unique_ptr<Schema> items;
  bool any = true;  // not a dict schema: accepts anything

  const Schema* prop(std::string_view k) const {
    for (const auto& p : props)
      if (p.first == k) return p.second.get();
    return nullptr;
  }

  static std::unique_ptr<Schema> compile(const Node* s) {
    auto out = std::make_unique<Schema>();
    if (!s || !s->is_obj()) return out;
    out->any = false;
    out->type = s->str("type");
    out->kind = out->type == "object"    ? Kind::Object
                : out->type == "array"   ? Kind::Array
                : out->type == "string"  ? Kind::String
                : out->type == "integer" ? Kind::Integer
                : out->type == "number"  ? Kind::Number
                : out->type == "boolean" ? Kind::Boolean
                                         : Kind::Any;
    if (const Node* v = s->getn("nullable")) out->nullable = v->t == T::True;
    if (const Node* v = s->getn("x-kubernetes-preserve-unknown-fields")) out->preserve = v->t == T::True;
    out->date_time = s->str("format") == "date-time";
    if (const Node* v = s->getn("enum")) {
      out->has_enum = true;
      if (v->is_arr()) out->enumv = v->a;
    }
    if (const Node* v = s->getn("minimum")) {
      if (v->t == T::Num) {
        out->has_min = true;
        out->min = std::strtod(v->s.c_str(), nullptr);
        out->min_lex = Ref(const_cast<Node*>(v));
      }
    }
    if (const Node* v = s->getn("maximum")) {
      if (v->t == T::Num) {
        out->has_max = true;
        out->max = std::strtod(v->s.c_str(), nullptr);
        out->max_lex = Ref(const_cast<Node*>(v));
      }
    }
    if (const Node* p = s->getn("properties")) {
      if (p->is_obj()) {
        out->has_props = true;
        for (const Member& m : p->o) {
          out->props.emplace_back(m.first, compile(m.second.get()));
          if (m.second->is_obj())
            if (const Ref* d = m.second->get("default")) out->defaults.emplace_back(m.first, *d);
        }
      }
    }
    if (const Node* r = s->getn("required"))
      if (r->is_arr())
        for (const Ref& x : r->a)
          if (x->is_str()) out->required.push_back(S(x->s));
    if (const Node* a = s->getn("additionalProperties")) {
      if (a->is_obj()) out->addl = compile(a);
      else if (a->t == T::True) out->addl_true = true;
    }
    if (const Node* it = s->getn("items"))
      if (it->is_obj()) out->items = compile(it);
    return out;
  }

  bool type_ok(const Node* v) const {
    switch (kind) {
      case Kind::Object: return v->t == T::Obj;
      case Kind::Array: return v->t == T::Arr;
      case Kind::String: return v->t == T::Str;
      case Kind::Integer: return v->t == T::Num && num_is_integral(v);
      case Kind::Number: return v->t == T::Num;
      case Kind::Boolean: return v->t == T::True || v->t == T::False;
      default: return true;  // no type, or one admission does not check
    }
  }

  // One pass: prune unknown fields, fill defaults (only on nodes not yet admitted: fresh,
  // private), and check.  Subtrees already admitted (shared with the stored object at the same
  // path) are skipped: CRD validation ratcheting taken to its conclusion, as in schema.py.
  // `changed`: set when this node or one below it was pruned or defaulted; an ancestor then drops
  // the bytes it may carry from the request body (jdom::Parser keeps them as its encoding)
  bool admit(Node* v, bool root, bool* changed = nullptr) const {
    bool dummy = false;
    if (!changed) changed = &dummy;
    if (any) return true;
    if (v->t == T::Null) return nullable || root || type.empty();
    if (v->admitted) return true;
    if (!type_ok(v)) return false;
    bool ok = true;
    if (has_enum) {
      bool hit = false;
      for (const Ref& e : enumv)
        if (jdom::equal(e.get(), v)) {
          hit = true;
          break;
        }
      if (!hit) ok = false;
    }
    if (date_time && v->t == T::Str && !is_date_time(v->s)) ok = false;
    if ((has_min || has_max) && v->t == T::Num) {
      const double d = std::strtod(v->s.c_str(), nullptr);
      if (has_min && d < min) ok = false;
      if (has_max && d > max) ok = false;
    }
    bool mine = false;
    if (v->t == T::Obj) {
      const bool keep_unknown = preserve || (!has_props && !addl && !addl_true);
      if (!keep_unknown && !addl && !addl_true) {
        for (size_t i = 0; i < v->o.size();) {
          const jdom::jstr& k = v->o[i].first;
          if (prop(k) || (root && (k == "apiVersion" || k == "kind" || k == "metadata"))) {
            ++i;
            continue;
          }
          v->o.erase(v->o.begin() + static_cast<long>(i));
          mine = true;
        }
      }
      for (const auto& d : defaults)
        if (!v->get(d.first)) {
          v->o.emplace_back(d.first, jdom::deep_copy(d.second.get()));
          mine = true;
        }
      for (const auto& r : required)
        if (!v->get(r)) ok = false;
      for (const Member& m : v->o) {
        if (root && m.first == "metadata") continue;
        const Schema* sub = prop(m.first);
        if (sub) {
          if (!sub->admit(m.second.get(), false, &mine)) ok = false;
        } else if (addl) {
          if (!addl->admit(m.second.get(), false, &mine)) ok = false;
        }
      }
    } else if (v->t == T::Arr && items) {
      for (const Ref& it : v->a)
        if (!items->admit(it.get(), false, &mine)) ok = false;
    }
    if (mine) {
      v->enc.clear();
      *changed = true;
    }
    return ok;
  }

  // the field errors of an object admit() refused (schema.py validate(): same messages)
  void errors(const Node* v, const std::string& path, std::vector<Ref>* out, bool root) const {
    if (any) return;
    const std::string fld = path.empty() ? "<root>" : path;
    auto cause = [&](const std::string& field, const char* reason, const std::string& msg) {
      Ref c = jdom::mk_obj();
      c->o.emplace_back("field", jdom::mk_str(field));
      c->o.emplace_back("reason", jdom::mk_str(reason));
      c->o.emplace_back("message", jdom::mk_str(msg));
      out->push_back(c);
    };
    if (v->t == T::Null) {
      if (nullable) return;
      if (!type.empty() && !root)
        cause(fld, "FieldValueTypeInvalid",
              "Invalid value: \"null\": " + fld + " in body must be of type " + type + ": \"null\"");
      return;
    }
    if (!type_ok(v)) {
      const std::string gt = go_type_name(v);
      cause(fld, "FieldValueTypeInvalid",
            "Invalid value: \"" + gt + "\": " + fld + " in body must be of type " + type + ": \"" + gt + "\"");
      return;
    }
    auto lex = [](const Node* n) { return n->t == T::Str ? S(n->s) : jdom::dump(const_cast<Node*>(n), 0); };
    if (has_enum) {
      bool hit = false;
      for (const Ref& e : enumv)
        if (jdom::equal(e.get(), v)) hit = true;
      if (!hit) {
        std::string allowed;
        for (size_t i = 0; i < enumv.size(); ++i) {
          if (i) allowed += ", ";
          allowed += "\"" + lex(enumv[i].get()) + "\"";
        }
        cause(fld, "FieldValueNotSupported", "Unsupported value: \"" + lex(v) + "\": supported values: " + allowed);
      }
    }
    if (date_time && v->t == T::Str && !is_date_time(v->s))
      cause(fld, "FieldValueInvalid",
            "Invalid value: \"" + S(v->s) + "\": " + fld + " in body must be of type date-time: \"" + S(v->s) + "\"");
    if (v->t == T::Num) {
      const double d = std::strtod(v->s.c_str(), nullptr);
      if (has_min && d < min)
        cause(fld, "FieldValueInvalid", "Invalid value: " + S(v->s) + ": " + fld +
                                            " in body should be greater than or equal to " + S(min_lex->s));
      if (has_max && d > max)
        cause(fld, "FieldValueInvalid", "Invalid value: " + S(v->s) + ": " + fld +
                                            " in body should be less than or equal to " + S(max_lex->s));
    }
    if (v->t == T::Obj) {
      for (const auto& r : required)
        if (!v->get(r)) cause(path.empty() ? r : path + "." + r, "FieldValueRequired", "Required value");
      for (const auto& p : props) {
        if (root && p.first == "metadata") continue;
        if (const Ref* x = v->get(p.first)) p.second->errors(x->get(), path.empty() ? p.first : path + "." + p.first,
                                                               out, false);
      }
      if (addl)
        for (const Member& m : v->o)
          if (!prop(m.first)) addl->errors(m.second.get(), path.empty() ? S(m.first) : path + "[" + S(m.first) + "]", out,
                                           false);
    } else if (v->t == T::Arr && items) {
      for (size_t i = 0; i < v->a.size(); ++i)
        items->errors(v->a[i].get(), path + "[" + std::to_string(i) + "]", out, false);
    }
  }
};

// ====================================================================== store

struct Watcher;
struct Conn;

// One event of the watch log.  The log keeps what a resuming watch needs -- the bytes the
// event carries and, for its scope, the object's (and for MODIFIED its previous version's)
// name, namespace and labels -- not the object trees: a superseded version is freed when the
// store replaces it, while its nodes are still in cache, instead of watch_window events later
// (when the log held the trees, the fixture's CPU per fire drifted with the heap's age).
// An object's scope: its metadata's name, namespace and labels, shared with the object (no
// allocation per event); a replay builds the {"metadata": {...}} a selector reads from it.
struct Scope {
  Ref name, ns, labels;
  bool set = false;  // a MODIFIED event's previous version, or none
};

struct Event {
  long long rv;
  int type;  // 0 ADDED 1 MODIFIED 2 DELETED
  Scope scope, old_scope;
  jdom::jstr bytes;  // the object as encoded in the event (pool-allocated: the log turns over FIFO)
  Ref held, held_old;  // APISERVERD_LOG_TREES=1 only: the trees too, as rounds 1-5 kept them (A/B arm)
};

const char* kEventType[] = {"ADDED", "MODIFIED", "DELETED"};

// objects of one (group, resource): shared by its served versions, as in server.py
struct Store {
  std::map<std::string, std::map<std::string, Ref>> data;  // namespace -> name -> stored object
  // label key -> value -> namespace -> names (built by the first LIST pinning key=value)
  std::unordered_map<std::string, std::unordered_map<std::string, std::map<std::string, std::set<std::string>>>> idx;
  std::deque<Event> log;
  long long floor = 0;
  std::vector<Watcher*> watchers;
};

struct Resource {
  std::string group, version, resource, kind, list_kind, singular, api_version;
  bool namespaced = true, status_sub = false, is_crd = false, virt = false;
  std::vector<std::string> short_names, verbs;
  std::unique_ptr<Schema> schema, status_schema;
  Ref schema_src;
  Store* store = nullptr;
};

const Node* labels_of(const Node* obj) {
  const Node* m = obj->getn("metadata");
  if (!m || !m->is_obj()) return nullptr;
  const Node* l = m->getn("labels");
  return (l && l->is_obj()) ? l : nullptr;
}

std::string_view meta_str(const Node* obj, const char* k) {
  const Node* m = obj->getn("metadata");
  if (!m || !m->is_obj()) return std::string_view();
  return m->str(k);
}

// ====================================================================== connections / watches

struct Request {
  std::string method, path, query_string, content_type, accept, authorization;
  std::vector<std::pair<std::string, std::string>> query;
  std::string raw_headers;  // the header lines as sent (the Python fallback parses them)
  std::string body;
  bool keep = true;

  const std::string* q(const char* k) const {
    for (const auto& kv : query)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  std::string qv(const char* k) const {
    const std::string* v = q(k);
    return v ? *v : std::string();
  }
};

struct Reply {
  int status = 200;
  Ref obj;  // a stored object: its cached bytes are the body (no copy through `body`)
  std::string body;
  std::string content_type = "application/json";
  std::string extra_headers;  // "Name: value\r\n"...
  bool watch = false;         // a watch started: the connection streams until it ends
};

struct Watcher {
  Conn* conn = nullptr;
  Resource* res = nullptr;
  std::string ns;  // "" = all namespaces
  Selector sel;
  bool bookmarks = false;
  bool ended = false;
  bool dirty = false;
  std::string pending;  // event lines before the response head went out (the initial replay)
  // once streaming, events go straight into the connection's buffer inside an open chunk whose
  // fixed-width size field (at chunk_at) is filled in when the chunk closes (end of the turn)
  bool streaming = false;
  size_t chunk_at = std::string::npos;
  uint64_t sent = 0;

  bool in_scope(const Node* obj) const {
    if (!ns.empty() && meta_str(obj, "namespace") != ns) return false;
    return sel.match(obj);
  }
};

struct Conn {
  int fd = -1;
  uint64_t id = 0;
  SSL* ssl = nullptr;
  bool handshaking = false;
  std::string in;
  std::string out;
  size_t out_off = 0;
  bool want_out = false;  // EPOLLOUT armed
  bool busy = false;      // a delayed reply or a watch holds the connection
  bool closed = false;
  bool close_after = false;
  bool continued = false;
  Watcher* watch = nullptr;
  bool watch_keep = true;  // the watch request's keep-alive: the connection serves on after it
  std::unique_ptr<Request> delayed;
};

struct Timer {
  double due;
  uint64_t seq;
  int kind;  // 0 delayed request, 1 watch timeout, 2 bookmarks
  uint64_t conn_id;
  bool operator>(const Timer& o) const { return due > o.due || (due == o.due && seq > o.seq); }
};

// CPU time of the calling thread (the server thread's phases: where the fixture's time goes)
long long thread_cpu_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return static_cast<long long>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

double mono() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + static_cast<double>(ts.tv_nsec) * 1e-9;
}

// ====================================================================== the server

#ifndef APISERVERD_STANDALONE
struct Server {
  PyObject_HEAD
  struct Impl* impl;
};
#endif

Ref subst(const Ref& t, const std::string& ph, const std::string& name);

struct Impl {
  std::recursive_mutex mu;
  long long now_ns = 0;
  long long rv = 0;
  size_t watch_window = 200000;
  std::mt19937_64 rng{std::random_device{}()};
  std::map<std::string, std::unique_ptr<Resource>> resources;  // "group/version/resource"
  std::vector<Resource*> order;                                 // registration order (discovery)
  std::map<std::string, std::unique_ptr<Store>> stores;        // "group/resource"
  std::map<std::string, double> latency;                       // verb -> s ("*": default)
  long long stats_total = 0;
  long long requests = 0;
  // server-thread CPU by phase (ns): socket reads + request parsing, verbs (route, store,
  // admission, encoding, watch fan-out), the Python fallback (/debug/fake controls), framing +
  // socket writes; and the loop's total
  // the server thread's time by phase, in TSC cycles (a thread-CPU clock read is a system call:
  // per request it cost more than the accounting is worth); the thread's CPU per turn scales them
  unsigned long long cyc_read = 0, cyc_verbs = 0, cyc_fallback = 0, cyc_write = 0, cyc_loop = 0;
  long long cpu_loop = 0;  // ns of thread CPU over the same turns as cyc_loop
  struct VerbKey {
    const Resource* ri;
    std::string verb, sub;
    bool operator<(const VerbKey& o) const {
      return std::tie(ri, verb, sub) < std::tie(o.ri, o.verb, o.sub);
    }
  };
  std::map<VerbKey, std::pair<unsigned long long, long long>> verb_cpu;  // -> (cycles, calls)
  std::pair<const VerbKey, std::pair<unsigned long long, long long>>* last_vk = nullptr;
  struct RecHash {
    size_t operator()(const std::pair<const Resource*, const char*>& p) const {
      return std::hash<const void*>()(p.first) * 1000003u ^ std::hash<const void*>()(p.second);
    }
  };
  std::unordered_map<std::pair<const Resource*, const char*>, long long, RecHash> rec_counts;
  // where a write's time goes, in TSC cycles (nested: `finish` includes `emit`)
  enum Ph { kParse, kMerge, kPrepare, kFinish, kEmit, kReply, kPhases };
  unsigned long long phase[kPhases] = {};
  struct PhaseTimer {
    unsigned long long* acc;
    unsigned long long t0;
    explicit PhaseTimer(unsigned long long* a) : acc(a), t0(__rdtsc()) {}
    ~PhaseTimer() { *acc += __rdtsc() - t0; }
  };
#ifndef APISERVERD_STANDALONE
  PyObject* fallback = nullptr;
#endif

  // event loop
  int epfd = -1, lfd = -1, evfd = -1;
  int port = 0;
  SSL_CTX* ssl_ctx = nullptr;
  std::thread thread;
  std::atomic<pid_t> loop_tid{0};  // the server thread's kernel id (the sampler's target)
  std::atomic<bool> stopping{false};
  bool running = false;
  double bookmark_interval = 60.0;
  uint64_t next_conn_id = 1;
  uint64_t timer_seq = 0;
  std::unordered_map<uint64_t, Conn*> conns;
  std::priority_queue<Timer, std::vector<Timer>, std::greater<Timer>> timers;
  std::vector<Watcher*> dirty_watchers;
  std::vector<Conn*> dirty_conns;
  // watch streams are flushed when the server has nothing else ready (or after kWatchDefer s):
  // under load one send carries many events instead of one send per event per turn
  // (APISERVERD_WATCH_DEFER_S overrides; 0 flushes every turn, as rounds 1-5 did)
  double watch_defer_s = 0.002;
  bool log_trees = false;  // APISERVERD_LOG_TREES=1: the log also holds the object trees (A/B)
  bool watch_deferred = false;
  double watch_defer_since = 0.0;
  long long sends = 0, turns = 0;
  // patch_unfinished with a per-turn budget: the harness's completion writes applied a few per
  // loop turn, between the turns that serve the other clients -- as a training operator's writes
  // interleave with everyone else's at a real apiserver -- instead of one batch that holds the
  // server (and every watch) for its whole length
  struct PendingPatches {
    std::string g, v, r;  // looked up each turn: a resource may go away meanwhile
    std::string sub, ph;
    Ref tree;
    std::vector<std::pair<std::string, std::string>> todo;  // (namespace, name)
    size_t next = 0, per_turn = 1;
  };
  std::deque<PendingPatches> pending_patches;
  long long pending_applied = 0;

  ~Impl() {
    for (auto& kv : conns) delete kv.second;
    if (ssl_ctx) SSL_CTX_free(ssl_ctx);
  }

  // ---------------------------------------------------------------- registry
  Resource* find(const std::string& g, const std::string& v, const std::string& r) {
    auto it = resources.find(g + "/" + v + "/" + r);
    return it == resources.end() ? nullptr : it->second.get();
  }

  Resource* add_resource(const std::string& g, const std::string& v, const std::string& r, const std::string& kind,
                         bool namespaced, bool status_sub, bool is_crd, bool virt, const std::string& singular,
                         const std::vector<std::string>& short_names, const std::vector<std::string>& verbs,
                         const Ref& schema) {
    auto res = std::make_unique<Resource>();
    res->group = g;
    res->version = v;
    res->resource = r;
    res->kind = kind;
    res->list_kind = kind + "List";
    res->singular = singular;
    res->api_version = g.empty() ? v : g + "/" + v;
    res->namespaced = namespaced;
    res->status_sub = status_sub;
    res->is_crd = is_crd;
    res->virt = virt;
    res->short_names = short_names;
    res->verbs = verbs.empty() ? std::vector<std::string>{"create", "delete", "deletecollection", "get", "list",
                                                          "patch", "update", "watch"}
                               : verbs;
    if (schema && schema->is_obj()) {
      res->schema_src = schema;
      res->schema = Schema::compile(schema.get());
      const Node* props = schema->getn("properties");
      const Node* st = (props && props->is_obj()) ? props->getn("status") : nullptr;
      if (st && st->is_obj()) res->status_schema = Schema::compile(st);
    }
    auto& st = stores[g + "/" + r];
    if (!st) st = std::make_unique<Store>();
    res->store = st.get();
    Resource* out = res.get();
    auto& slot = resources[g + "/" + v + "/" + r];
    if (slot) order.erase(std::remove(order.begin(), order.end(), slot.get()), order.end());
    slot = std::move(res);
    order.push_back(out);
    return out;
  }

  void builtins() {
    struct B {
      const char *g, *v, *r, *k;
      bool ns, st;
      std::vector<std::string> sn;
      bool virt;
    };
    const std::vector<B> bs = {
        {"", "v1", "namespaces", "Namespace", false, true, {}, false},
        {"", "v1", "pods", "Pod", true, true, {"po"}, false},
        {"", "v1", "events", "Event", true, false, {"ev"}, false},
        {"", "v1", "configmaps", "ConfigMap", true, false, {"cm"}, false},
        {"", "v1", "secrets", "Secret", true, false, {}, false},
        {"", "v1", "services", "Service", true, true, {"svc"}, false},
        {"", "v1", "serviceaccounts", "ServiceAccount", true, false, {"sa"}, false},
        {"coordination.k8s.io", "v1", "leases", "Lease", true, false, {}, false},
        {"batch", "v1", "jobs", "Job", true, true, {}, false},
        {"events.k8s.io", "v1", "events", "Event", true, false, {"ev"}, false},
        {"authentication.k8s.io", "v1", "tokenreviews", "TokenReview", false, false, {}, true},
        {"authorization.k8s.io", "v1", "subjectaccessreviews", "SubjectAccessReview", false, false, {}, true},
        {"apiextensions.k8s.io", "v1", "customresourcedefinitions", "CustomResourceDefinition", false, true,
         {"crd", "crds"}, false},
        {"rbac.authorization.k8s.io", "v1", "roles", "Role", true, false, {}, false},
        {"rbac.authorization.k8s.io", "v1", "rolebindings", "RoleBinding", true, false, {}, false},
        {"rbac.authorization.k8s.io", "v1", "clusterroles", "ClusterRole", false, false, {}, false},
        {"rbac.authorization.k8s.io", "v1", "clusterrolebindings", "ClusterRoleBinding", false, false, {}, false},
        {"apps", "v1", "deployments", "Deployment", true, true, {"deploy"}, false},
        {"networking.k8s.io", "v1", "networkpolicies", "NetworkPolicy", true, false, {"netpol"}, false},
    };
    for (const B& b : bs)
      add_resource(b.g, b.v, b.r, b.k, b.ns, b.st, false, b.virt, "", b.sn,
                   b.virt ? std::vector<std::string>{"create"} : std::vector<std::string>{}, Ref());
    for (const char* ns : {"default", "kube-system", "kube-public", "kube-node-lease"}) put_namespace(ns);
  }

  void put_namespace(const std::string& name) {
    Resource* ri = find("", "v1", "namespaces");
    Ref o = jdom::mk_obj();
    o->o.emplace_back("apiVersion", jdom::mk_str("v1"));
    o->o.emplace_back("kind", jdom::mk_str("Namespace"));
    Ref m = jdom::mk_obj();
    m->o.emplace_back("name", jdom::mk_str(name));
    m->o.emplace_back("uid", jdom::mk_str(uuid4(rng)));
    m->o.emplace_back("resourceVersion", jdom::mk_str(std::to_string(++rv)));
    m->o.emplace_back("creationTimestamp", jdom::mk_str(rfc3339(now_ns)));
    o->o.emplace_back("metadata", m);
    Ref spec = jdom::mk_obj();
    Ref fin = jdom::mk_arr();
    fin->a.push_back(jdom::mk_str("kubernetes"));
    spec->o.emplace_back("finalizers", fin);
    o->o.emplace_back("spec", spec);
    Ref st = jdom::mk_obj();
    st->o.emplace_back("phase", jdom::mk_str("Active"));
    o->o.emplace_back("status", st);
    put_raw(ri, "", o);
  }

  // the resources a CRD object serves (registry.py resources_from_crd) + Established status
  void on_crd_written(Node* crd) {
    const Node* spec = crd->getn("spec");
    if (!spec || !spec->is_obj()) return;
    const Node* names = spec->getn("names");
    const std::string group = S(spec->str("group"));
    const bool namespaced = spec->str("scope").empty() || spec->str("scope") == "Namespaced";
    std::string plural, kind, singular;
    std::vector<std::string> sn;
    if (names && names->is_obj()) {
      plural = names->str("plural");
      kind = names->str("kind");
      singular = names->str("singular");
      if (const Node* s = names->getn("shortNames"))
        if (s->is_arr())
          for (const Ref& x : s->a)
            if (x->is_str()) sn.push_back(S(x->s));
    }
    if (const Node* vs = spec->getn("versions"))
      if (vs->is_arr())
        for (const Ref& v : vs->a) {
          if (!v->is_obj()) continue;
          const Node* served = v->getn("served");
          if (served && served->t == T::False) continue;
          Ref schema;
          if (const Node* sc = v->getn("schema"))
            if (sc->is_obj())
              if (const Ref* oa = sc->get("openAPIV3Schema")) schema = *oa;
          const Node* subs = v->getn("subresources");
          const bool st = subs && subs->is_obj() && subs->get("status");
          add_resource(group, S(v->str("name")), plural, kind, namespaced, st, true, false, singular, sn, {}, schema);
        }
    // mark Established like the apiextensions controller
    Ref status = jdom::mk_obj();
    Ref conds = jdom::mk_arr();
    auto cond = [](const char* t, const char* reason) {
      Ref c = jdom::mk_obj();
      c->o.emplace_back("type", jdom::mk_str(t));
      c->o.emplace_back("status", jdom::mk_str("True"));
      c->o.emplace_back("reason", jdom::mk_str(reason));
      return c;
    };
    conds->a.push_back(cond("NamesAccepted", "NoConflicts"));
    conds->a.push_back(cond("Established", "InitialNamesAccepted"));
    status->o.emplace_back("conditions", conds);
    status->o.emplace_back("acceptedNames", (names && names->is_obj()) ? jdom::shallow(names) : jdom::mk_obj());
    crd->set("status", status);
  }

  // ---------------------------------------------------------------- store primitives
  Ref get_raw(Resource* ri, const std::string& ns, const std::string& name) {
    auto& d = ri->store->data;
    auto it = d.find(ri->namespaced ? ns : std::string());
    if (it == d.end()) return Ref();
    auto jt = it->second.find(name);
    return jt == it->second.end() ? Ref() : jt->second;
  }

  static void reindex(Store* st, const std::string& ns, const std::string& name, const Node* old, const Node* neu) {
    if (st->idx.empty()) return;
    const Node* ol = old ? labels_of(old) : nullptr;
    const Node* nl = neu ? labels_of(neu) : nullptr;
    if (old && neu && (ol == nl || (ol && nl && jdom::equal(ol, nl)))) return;
    for (auto& kv : st->idx) {
      const jdom::jstr* ov = ol ? Selector::label(ol, kv.first) : nullptr;
      const jdom::jstr* nv = nl ? Selector::label(nl, kv.first) : nullptr;
      if (old && neu && ((!ov && !nv) || (ov && nv && *ov == *nv))) continue;
      if (ov) {
        auto a = kv.second.find(S(*ov));
        if (a != kv.second.end()) {
          auto b = a->second.find(ns);
          if (b != a->second.end()) b->second.erase(name);
        }
      }
      if (nv) kv.second[S(*nv)][ns].insert(name);
    }
  }

  void put_raw(Resource* ri, const std::string& ns_in, const Ref& obj) {
    const std::string ns = ri->namespaced ? ns_in : std::string();
    const std::string name = S(meta_str(obj.get(), "name"));
    auto& slot = ri->store->data[ns][name];
    Ref old = slot;
    slot = obj;
    reindex(ri->store, ns, name, old.get(), obj.get());
  }

  size_t count(Resource* ri, const std::string* ns) {
    size_t n = 0;
    for (auto& kv : ri->store->data)
      if (!ns || kv.first == *ns) n += kv.second.size();
    return n;
  }

  void record(const char* verb, const Resource* ri) {
    ++rec_counts[{ri, verb}];
    ++stats_total;
  }

  // ---------------------------------------------------------------- watch fan-out
  // where a watcher's next event line goes: its pending buffer, or the open chunk
  std::string& event_sink(Watcher* w) {
    if (!w->streaming || !w->conn || w->conn->closed) return w->pending;
    std::string& o = w->conn->out;
    if (w->chunk_at == std::string::npos) {
      w->chunk_at = o.size();
      o.append("00000000\r\n");  // chunk-size, leading zeros allowed (RFC 9112 7.1)
    }
    return o;
  }

  void put_event(Watcher* w, int type, std::string_view obj) {
    if (w->ended) return;
    ++w->sent;
    std::string& p = event_sink(w);
    p.append("{\"type\":\"");
    p.append(kEventType[type]);
    p.append("\",\"object\":");
    p.append(obj.data(), obj.size());
    p.append("}\n");
    if (!w->dirty) {
      w->dirty = true;
      dirty_watchers.push_back(w);
    }
  }
  void put_event(Watcher* w, int type, Node* obj) {
    const jdom::jstr& e = jdom::encoded(obj);
    put_event(w, type, std::string_view(e));
  }

  // a MODIFIED that moves an object into or out of a watcher's scope is an ADDED / DELETED
  void offer(Watcher* w, int type, std::string_view obj, bool modified_with_old, bool now_in, bool was_in) {
    if (type == 1 && modified_with_old) {
      if (was_in && !now_in) put_event(w, 2, obj);
      else if (now_in && !was_in) put_event(w, 0, obj);
      else if (now_in) put_event(w, 1, obj);
      return;
    }
    if (now_in) put_event(w, type, obj);
  }

  // what a resuming watcher's scope reads of an object: its name, namespace and labels
  static Scope scope_of(const Node* obj) {
    Scope sc;
    sc.set = true;
    const Node* m = obj->getn("metadata");
    if (m && m->is_obj()) {
      if (const Ref* v = m->get("name")) sc.name = *v;
      if (const Ref* v = m->get("namespace")) sc.ns = *v;
      if (const Ref* v = m->get("labels")) sc.labels = *v;
    }
    return sc;
  }
  // ... as the object a selector matches (a replay only)
  static Ref scope_tree(const Scope& sc) {
    Ref t = jdom::mk_obj();
    Ref mm = jdom::mk_obj();
    if (sc.name) mm->o.emplace_back("name", sc.name);
    if (sc.ns) mm->o.emplace_back("namespace", sc.ns);
    if (sc.labels) mm->o.emplace_back("labels", sc.labels);
    t->o.emplace_back("metadata", mm);
    return t;
  }

  void emit(Resource* ri, int type, const Ref& obj, const Ref& old, long long at) {
    PhaseTimer pt(&phase[kEmit]);
    Store* st = ri->store;
    const jdom::jstr& enc = jdom::encoded(obj.get());
    const bool with_old = type == 1 && old;
    st->log.push_back(Event{at, type, scope_of(obj.get()), with_old ? scope_of(old.get()) : Scope(),
                            jdom::jstr(enc.data(), enc.size()),
                            log_trees ? obj : Ref(), log_trees ? old : Ref()});
    while (st->log.size() > watch_window) {
      st->floor = st->log.front().rv;
      st->log.pop_front();
    }
    if (st->watchers.empty()) return;
    const bool modified = type == 1 && old;
    bool same_scope = false;
    if (modified) {
      const Node* om = old->getn("metadata");
      const Node* nm = obj->getn("metadata");
      if (om && nm) {
        const Node* ol = om->getn("labels");
        const Node* nl = nm->getn("labels");
        same_scope = (ol == nl || (ol && nl && jdom::equal(ol, nl)) || (!ol && !nl)) &&
                     om->str("namespace") == nm->str("namespace");
      }
    }
    const std::string_view bytes(enc);
    for (Watcher* w : st->watchers) {
      if (w->ended) continue;
      const bool now_in = w->in_scope(obj.get());
      bool was_in = false;
      if (modified) was_in = (same_scope && w->sel.labels_only) ? now_in : w->in_scope(old.get());
      if (now_in || was_in) offer(w, type, bytes, with_old, now_in, was_in);
    }
  }

  // ---------------------------------------------------------------- admission
  long long slow_admits = 0;
  bool admit_object(Resource* ri, Node* obj, const std::string& name, ApiErr* err) {
    if (!ri->schema) return true;
    if (ri->schema->admit(obj, true)) return true;
    ++slow_admits;
    std::vector<Ref> causes;
    ri->schema->errors(obj, "", &causes, true);
    if (causes.empty()) return true;  // admit() pruned/defaulted its way to a valid object
    *err = invalid(ri, name, causes);
    return false;
  }

  bool admit_status(Resource* ri, Node* status, const std::string& name, ApiErr* err) {
    if (!ri->status_schema) return true;
    if (ri->status_schema->admit(status, false)) return true;
    ++slow_admits;
    std::vector<Ref> causes;
    ri->status_schema->errors(status, "status", &causes, false);
    if (causes.empty()) return true;
    *err = invalid(ri, name, causes);
    return false;
  }

  static ApiErr invalid(Resource* ri, const std::string& name, const std::vector<Ref>& causes) {
    std::string msg;
    for (size_t i = 0; i < causes.size(); ++i) {
      if (i) msg += "; ";
      msg += S(causes[i]->str("field")) + ": " + S(causes[i]->str("message"));
    }
    ApiErr e = mkerr(422, "Invalid", ri->group.empty() ? ri->kind + " \"" + name + "\" is invalid: " + msg
                                                       : ri->kind + "." + ri->group + " \"" + name +
                                                             "\" is invalid: " + msg);
    Ref d = name_details(name, ri->group, ri->kind);
    Ref arr = jdom::mk_arr();
    arr->a.assign(causes.begin(), causes.end());
    d->o.emplace_back("causes", arr);
    e.details = d;
    return e;
  }

  static bool valid_name(const std::string& n) {
    if (n.empty() || n.size() > 253) return false;
    for (char c : n)
      if (!((c >= 'a' && c <= 'z') || (c >= '0' && c <= '9') || c == '-' || c == '.')) return false;
    auto alnum = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    return alnum(n.front()) && alnum(n.back());
  }

  // ---------------------------------------------------------------- verbs
  // Each returns the stored object (or an error): the caller serialises it.

  Ref v_get(Resource* ri, const std::string& ns, const std::string& name, ApiErr* err) {
    record("get", ri);
    Ref o = get_raw(ri, ns, name);
    if (!o) *err = not_found(ri->resource, ri->group, name);
    return o;
  }

  bool check_namespace(Resource* ri, const std::string& ns, ApiErr* err) {
    if (!ri->namespaced) return true;
    if (ns.empty()) {
      *err = bad_request("an empty namespace may not be set during creation");
      return false;
    }
    if (!get_raw(find("", "v1", "namespaces"), "", ns)) {
      *err = not_found("namespaces", "", ns);
      return false;
    }
    return true;
  }

  Ref v_create(Resource* ri, const std::string& url_ns, Ref body, bool dry_run, ApiErr* err) {
    record("create", ri);
    Node* b = body.get();
    Ref meta;
    if (const Ref* m = b->get("metadata"); m && (*m)->is_obj()) {
      meta = *m;
    } else {
      meta = jdom::mk_obj();
      b->set("metadata", meta);
    }
    Node* m = meta.get();
    std::string ns = url_ns;
    if (ri->namespaced) {
      const std::string bns = S(m->str("namespace"));
      if (!bns.empty() && !ns.empty() && bns != ns) {
        *err = bad_request("the namespace of the provided object does not match the namespace sent on the request");
        return Ref();
      }
      if (ns.empty()) ns = bns;
      m->set("namespace", jdom::mk_str(ns));
    } else {
      m->erase("namespace");
      ns.clear();
    }
    if (ri->virt) return review(ri, body);
    b->set("apiVersion", jdom::mk_str(ri->api_version));
    b->set("kind", jdom::mk_str(ri->kind));
    std::string name = S(m->str("name"));
    if (name.empty() && !m->str("generateName").empty()) {
      static const char chars[] = "bcdfghjklmnpqrstvwxz2456789";
      for (int i = 0; i < 16; ++i) {
        std::string cand = S(m->str("generateName"));
        for (int j = 0; j < 5; ++j) cand.push_back(chars[rng() % (sizeof(chars) - 1)]);
        if (!get_raw(ri, ns, cand)) {
          name = cand;
          break;
        }
      }
      m->set("name", jdom::mk_str(name));
    }
    if (name.empty()) {
      Ref c = jdom::mk_obj();
      c->o.emplace_back("field", jdom::mk_str("metadata.name"));
      c->o.emplace_back("reason", jdom::mk_str("FieldValueRequired"));
      c->o.emplace_back("message", jdom::mk_str("Required value: name or generateName is required"));
      *err = invalid(ri, name, {c});
      return Ref();
    }
    if (!valid_name(name) && ri->kind != "Event") {
      Ref c = jdom::mk_obj();
      c->o.emplace_back("field", jdom::mk_str("metadata.name"));
      c->o.emplace_back("reason", jdom::mk_str("FieldValueInvalid"));
      c->o.emplace_back("message", jdom::mk_str("Invalid value: \"" + name +
                                                "\": a lowercase RFC 1123 subdomain must consist of lower case "
                                                "alphanumeric characters, '-' or '.', and must start and end with an "
                                                "alphanumeric character"));
      *err = invalid(ri, name, {c});
      return Ref();
    }
    if (!check_namespace(ri, ns, err)) return Ref();
    if (get_raw(ri, ns, name)) {
      *err = already_exists(ri->resource, ri->group, name);
      return Ref();
    }
    if (ri->status_sub && ri->is_crd) b->erase("status");
    if (!admit_object(ri, b, name, err)) return Ref();
    for (const char* k : {"resourceVersion", "deletionTimestamp", "deletionGracePeriodSeconds", "selfLink"})
      m->erase(k);
    m->set("uid", jdom::mk_str(uuid4(rng)));
    m->set("creationTimestamp", jdom::mk_str(rfc3339(now_ns)));
    m->set("generation", jdom::mk_num(1));
    if (dry_run) return body;
    const long long at = ++rv;
    m->set("resourceVersion", jdom::mk_str(std::to_string(at)));
    if (ri->kind == "CustomResourceDefinition") on_crd_written(b);
    if (ri->schema) jdom::mark_admitted(b);
    put_raw(ri, ns, body);
    emit(ri, 0, body, Ref(), at);
    return body;
  }

  Ref review(Resource* ri, Ref body) {
    body->set("apiVersion", jdom::mk_str(ri->api_version));
    body->set("kind", jdom::mk_str(ri->kind));
    Ref st = jdom::mk_obj();
    if (ri->kind == "TokenReview") {
      st->o.emplace_back("authenticated", jdom::mk_bool(false));
      st->o.emplace_back("user", jdom::mk_obj());
    } else {
      st->o.emplace_back("allowed", jdom::mk_bool(true));
    }
    body->set("status", st);
    return body;
  }

  // store `neu` unless it equals `old` (server.py _finish_write); `nm`: neu's private metadata
  Ref finish_write(Resource* ri, const std::string& ns, const std::string& name, const Ref& old, Ref neu, Node* nm,
                   ApiErr* err) {
    nm->set("resourceVersion", jdom::mk_str(meta_str(old.get(), "resourceVersion")));
    if (jdom::equal(old.get(), neu.get())) return old;
    const Node* dts = nm->getn("deletionTimestamp");
    const Node* fin = nm->getn("finalizers");
    const bool has_dts = dts && !(dts->t == T::Null || (dts->t == T::Str && dts->s.empty()));
    const bool has_fin = fin && fin->is_arr() && !fin->a.empty();
    if (has_dts && !has_fin) return remove(ri, ns, name, old);
    const long long at = ++rv;
    nm->set("resourceVersion", jdom::mk_str(std::to_string(at)));
    if (ri->kind == "CustomResourceDefinition") on_crd_written(neu.get());
    if (ri->schema) jdom::mark_admitted(neu.get());
    put_raw(ri, ns, neu);
    emit(ri, 1, neu, old, at);
    (void)err;
    return neu;
  }

  // server.py _prepare_update; returns neu with a private metadata node in *nm_out
  Ref prepare_update(Resource* ri, const Ref& old, Ref body, const std::string& sub, Node** nm_out, ApiErr* err) {
    const Node* om = old->getn("metadata");
    if (sub == "status") {
      Ref neu = jdom::shallow(old.get());
      Ref nm = jdom::shallow(om);
      neu->set("metadata", nm);
      if (const Ref* st = body->get("status")) {
        neu->set("status", *st);
      } else {
        neu->erase("status");
      }
      if (ri->schema) {
        const Ref* st = neu->get("status");
        if (st && (*st)->t != T::Null && !admit_status(ri, st->get(), S(om->str("name")), err)) return Ref();
      }
      *nm_out = nm.get();
      return neu;
    }
    if (!sub.empty()) {
      *err = mkerr(404, "NotFound", "the server could not find the requested resource (" + sub + ")");
      return Ref();
    }
    Ref neu = body;
    neu->set("apiVersion", jdom::mk_str(ri->api_version));
    neu->set("kind", jdom::mk_str(ri->kind));
    Ref nm;
    if (const Ref* m = neu->get("metadata"); m && (*m)->is_obj()) {
      nm = jdom::shallow(m->get());
    } else {
      nm = jdom::mk_obj();
    }
    neu->set("metadata", nm);
    for (const char* k : {"uid", "creationTimestamp", "namespace", "name", "generation", "deletionTimestamp",
                          "deletionGracePeriodSeconds"}) {
      if (const Ref* v = om->get(k)) nm->set(k, *v);
      else nm->erase(k);
    }
    if (ri->status_sub) {
      if (const Ref* st = old->get("status")) neu->set("status", *st);
      else neu->erase("status");
    }
    if (!admit_object(ri, neu.get(), S(om->str("name")), err)) return Ref();
    bool spec_changed = false;
    auto skip = [](std::string_view k) {
      return k == "metadata" || k == "status" || k == "apiVersion" || k == "kind";
    };
    for (const Member& mm : old->o)
      if (!skip(mm.first)) {
        const Ref* nv = neu->get(mm.first);
        if (!nv || !jdom::equal(mm.second.get(), nv->get())) spec_changed = true;
      }
    for (const Member& mm : neu->o)
      if (!skip(mm.first) && !old->get(std::string_view(mm.first))) spec_changed = true;
    if (spec_changed) {
      long long g = 1;
      if (const Node* gv = om->getn("generation"))
        if (gv->t == T::Num) g = std::strtoll(gv->s.c_str(), nullptr, 10);
      nm->set("generation", jdom::mk_num(g + 1));
    }
    *nm_out = nm.get();
    return neu;
  }

  Ref v_update(Resource* ri, const std::string& ns_in, const std::string& name, Ref body, const std::string& sub,
               ApiErr* err) {
    record("update", ri);
    const std::string ns = ri->namespaced ? ns_in : std::string();
    Ref old = get_raw(ri, ns, name);
    const Node* bm = body->getn("metadata");
    if (bm && bm->is_obj() && !bm->str("name").empty() && bm->str("name") != name) {
      *err = bad_request("the name of the object does not match the name on the URL");
      return Ref();
    }
    if (!old) {
      *err = not_found(ri->resource, ri->group, name);
      return Ref();
    }
    const std::string_view brv = (bm && bm->is_obj()) ? bm->str("resourceVersion") : std::string_view();
    if (!brv.empty() && brv != meta_str(old.get(), "resourceVersion")) {
      *err = conflict(ri->resource, ri->group, name, kModified);
      return Ref();
    }
    Node* nm = nullptr;
    Ref neu = prepare_update(ri, old, body, sub, &nm, err);
    if (!neu) return Ref();
    return finish_write(ri, ns, name, old, neu, nm, err);
  }

  Ref v_patch(Resource* ri, const std::string& ns_in, const std::string& name, Ref patch, const std::string& ptype,
              const std::string& sub, ApiErr* err) {
    record("patch", ri);
    const std::string ns = ri->namespaced ? ns_in : std::string();
    Ref old = get_raw(ri, ns, name);
    if (!old) {
      *err = not_found(ri->resource, ri->group, name);
      return Ref();
    }
    if (ptype == "strategic" && ri->is_crd) {
      *err = mkerr(415, "UnsupportedMediaType",
                   "the body of the request was in an unknown format - accepted media types include: "
                   "application/json-patch+json, application/merge-patch+json");
      return Ref();
    }
    if (!patch->is_obj()) {
      *err = bad_request("merge patch must be a JSON object");
      return Ref();
    }
    const Node* pm = patch->getn("metadata");
    const std::string_view prv = (pm && pm->is_obj()) ? pm->str("resourceVersion") : std::string_view();
    if (!prv.empty() && prv != meta_str(old.get(), "resourceVersion")) {
      *err = conflict(ri->resource, ri->group, name, kModified);
      return Ref();
    }
    Ref merged;
    {
      PhaseTimer pt(&phase[kMerge]);
      merged = jdom::merge_patch(old, patch);
    }
    Node* nm = nullptr;
    Ref neu;
    {
      PhaseTimer pt(&phase[kPrepare]);
      neu = prepare_update(ri, old, merged, sub, &nm, err);
    }
    if (!neu) return Ref();
    PhaseTimer pt(&phase[kFinish]);
    return finish_write(ri, ns, name, old, neu, nm, err);
  }

  Ref remove(Resource* ri, const std::string& ns, const std::string& name, const Ref& old) {
    auto& d = ri->store->data;
    auto it = d.find(ri->namespaced ? ns : std::string());
    if (it != d.end()) it->second.erase(name);
    reindex(ri->store, ri->namespaced ? ns : std::string(), name, old.get(), nullptr);
    const long long at = ++rv;
    Ref gone = jdom::shallow(old.get());
    Ref gm = jdom::shallow(old->getn("metadata"));
    gm->set("resourceVersion", jdom::mk_str(std::to_string(at)));
    gone->set("metadata", gm);
    emit(ri, 2, gone, Ref(), at);
    return gone;
  }

  Ref v_delete(Resource* ri, const std::string& ns_in, const std::string& name, const std::string& policy,
               const Node* pre, ApiErr* err) {
    record("delete", ri);
    const std::string ns = ri->namespaced ? ns_in : std::string();
    Ref old = get_raw(ri, ns, name);
    if (!old) {
      *err = not_found(ri->resource, ri->group, name);
      return Ref();
    }
    const Node* om = old->getn("metadata");
    if (pre && pre->is_obj()) {
      const std::string puid = S(pre->str("uid"));
      if (!puid.empty() && puid != om->str("uid")) {
        *err = conflict(ri->resource, ri->group, name, "Precondition failed: UID in precondition: " + puid +
                                                           ", UID in object meta: " + S(om->str("uid")));
        return Ref();
      }
      const std::string_view prv = pre->str("resourceVersion");
      if (!prv.empty() && prv != om->str("resourceVersion")) {
        *err = conflict(ri->resource, ri->group, name, "Precondition failed: ResourceVersion mismatch");
        return Ref();
      }
    }
    (void)policy;  // no ownerReference GC natively (server.py gc=True runs on the Python server)
    const Node* fin = om->getn("finalizers");
    if (fin && fin->is_arr() && !fin->a.empty()) {
      const Node* dts = om->getn("deletionTimestamp");
      if (dts && dts->t == T::Str && !dts->s.empty()) return old;
      Ref neu = jdom::shallow(old.get());
      Ref nm = jdom::shallow(om);
      nm->set("deletionTimestamp", jdom::mk_str(rfc3339(now_ns)));
      nm->set("deletionGracePeriodSeconds", jdom::mk_num(0));
      const long long at = ++rv;
      nm->set("resourceVersion", jdom::mk_str(std::to_string(at)));
      neu->set("metadata", nm);
      put_raw(ri, ns, neu);
      emit(ri, 1, neu, old, at);
      return neu;
    }
    return remove(ri, ns, name, old);
  }

  // LIST; writes the response body into *out
  bool v_list(Resource* ri, const std::string& ns, const Selector& sel, long long limit, const std::string& cont,
              std::string* out, ApiErr* err) {
    record("list", ri);
    Store* st = ri->store;
    std::string start_after;
    long long list_rv = rv;
    if (!cont.empty()) {
      std::string raw;
      Ref tok;
      if (b64url_decode(cont, &raw)) tok = jdom::parse(raw.data(), raw.size());
      const Node* k = tok && tok->is_obj() ? tok->getn("k") : nullptr;
      const Node* r = tok && tok->is_obj() ? tok->getn("rv") : nullptr;
      if (!k || !k->is_str() || !r || r->t != T::Num) {
        *err = bad_request("invalid continue token");
        return false;
      }
      start_after = k->s;
      list_rv = std::strtoll(r->s.c_str(), nullptr, 10);
    }
    // namespaces to scan
    std::vector<std::string> spaces;
    if (ri->namespaced && !ns.empty()) {
      spaces.push_back(ns);
    } else {
      for (auto& kv : st->data) spaces.push_back(kv.first);
    }
    const std::map<std::string, std::set<std::string>>* by_ns = nullptr;
    if (sel.pinned) {
      auto it = st->idx.find(sel.pin_key);
      if (it == st->idx.end()) {
        auto& by_val = st->idx[sel.pin_key];
        for (auto& nsk : st->data)
          for (auto& ob : nsk.second) {
            const jdom::jstr* v = Selector::label(labels_of(ob.second.get()), sel.pin_key);
            if (v) by_val[S(*v)][nsk.first].insert(ob.first);
          }
        it = st->idx.find(sel.pin_key);
      }
      static const std::map<std::string, std::set<std::string>> none;
      auto vit = it->second.find(sel.pin_val);
      by_ns = vit == it->second.end() ? &none : &vit->second;
    }
    out->append("{\"apiVersion\":");
    jdom::put_string(out, ri->api_version);
    out->append(",\"kind\":");
    jdom::put_string(out, ri->list_kind);
    out->append(",\"metadata\":{\"resourceVersion\":\"");
    out->append(std::to_string(list_rv));
    out->append("\"");
    std::string items;
    items.reserve(4096);
    long long n = 0;
    std::string more, last_key;
    bool first = true;
    for (const std::string& s : spaces) {
      auto dit = st->data.find(s);
      if (dit == st->data.end()) continue;
      auto visit = [&](const std::string& name, const Ref& obj) -> bool {
        if (!start_after.empty() && s + "/" + name <= start_after) return true;
        if (!sel.match(obj.get())) return true;
        if (limit > 0 && n >= limit) {
          more = s + "/" + name;
          return false;
        }
        if (!first) items.push_back(',');
        first = false;
        jdom::write(&items, obj.get());
        last_key = S(meta_str(obj.get(), "namespace")) + "/" + name;
        ++n;
        return true;
      };
      bool go = true;
      if (by_ns) {
        auto nit = by_ns->find(s);
        if (nit == by_ns->end()) continue;
        for (const std::string& name : nit->second) {
          auto oit = dit->second.find(name);
          if (oit == dit->second.end()) continue;
          if (!(go = visit(name, oit->second))) break;
        }
      } else {
        for (auto& ob : dit->second)
          if (!(go = visit(ob.first, ob.second))) break;
      }
      if (!go) break;
    }
    if (!more.empty()) {
      std::string tok = "{\"k\":";
      jdom::put_string(&tok, last_key);
      tok += ",\"rv\":" + std::to_string(list_rv) + "}";
      out->append(",\"continue\":\"");
      out->append(b64url_encode(tok));
      out->append("\",\"remainingItemCount\":0");
    }
    out->append("},\"items\":[");
    out->append(items);
    out->append("]}");
    return true;
  }

  // ---------------------------------------------------------------- discovery
  std::string discovery_entry(Resource* r) {
    std::string o = "{\"name\":";
    jdom::put_string(&o, r->resource);
    o += ",\"singularName\":";
    std::string sing = r->singular;
    if (sing.empty()) {
      sing = r->kind;
      for (auto& c : sing) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    }
    jdom::put_string(&o, sing);
    o += ",\"namespaced\":";
    o += r->namespaced ? "true" : "false";
    o += ",\"kind\":";
    jdom::put_string(&o, r->kind);
    o += ",\"verbs\":[";
    for (size_t i = 0; i < r->verbs.size(); ++i) {
      if (i) o += ",";
      jdom::put_string(&o, r->verbs[i]);
    }
    o += "]";
    if (!r->short_names.empty()) {
      o += ",\"shortNames\":[";
      for (size_t i = 0; i < r->short_names.size(); ++i) {
        if (i) o += ",";
        jdom::put_string(&o, r->short_names[i]);
      }
      o += "]";
    }
    o += "}";
    return o;
  }

  bool discovery(const std::string& path, Reply* rep) {
    if (path == "/healthz" || path == "/readyz" || path == "/livez") {
      rep->body = "ok";
      rep->content_type = "text/plain";
      return true;
    }
    if (path == "/version") {
      rep->body = "{\"major\":\"1\",\"minor\":\"34\",\"gitVersion\":\"v1.34.0-cron-operator-amd-fake\","
                  "\"platform\":\"linux/amd64\"}";
      return true;
    }
    if (path == "/api") {
      rep->body = "{\"kind\":\"APIVersions\",\"versions\":[\"v1\"]}";
      return true;
    }
    if (path == "/api/v1") {
      std::string o = "{\"kind\":\"APIResourceList\",\"apiVersion\":\"v1\",\"groupVersion\":\"v1\",\"resources\":[";
      bool first = true;
      for (Resource* r : order)
        if (r->group.empty()) {
          if (!first) o += ",";
          first = false;
          o += discovery_entry(r);
        }
      rep->body = o + "]}";
      return true;
    }
    if (path == "/apis") {
      std::map<std::string, std::vector<std::string>> groups;
      for (const Resource* r : order) {
        if (r->group.empty()) continue;
        auto& vs = groups[r->group];
        if (std::find(vs.begin(), vs.end(), r->version) == vs.end()) vs.push_back(r->version);
      }
      std::string o = "{\"kind\":\"APIGroupList\",\"apiVersion\":\"v1\",\"groups\":[";
      bool first = true;
      for (auto& g : groups) {
        if (!first) o += ",";
        first = false;
        o += "{\"name\":";
        jdom::put_string(&o, g.first);
        o += ",\"versions\":[";
        std::string last;
        for (size_t i = 0; i < g.second.size(); ++i) {
          if (i) o += ",";
          last = "{\"groupVersion\":\"" + g.first + "/" + g.second[i] + "\",\"version\":\"" + g.second[i] + "\"}";
          o += last;
        }
        o += "],\"preferredVersion\":" + last + "}";
      }
      rep->body = o + "]}";
      return true;
    }
    return false;
  }

  // ---------------------------------------------------------------- request handling
  static std::vector<std::string> split_path(const std::string& p) {
    std::vector<std::string> parts;
    size_t i = 0;
    while (i < p.size()) {
      while (i < p.size() && p[i] == '/') ++i;
      if (i >= p.size()) break;
      const size_t j = p.find('/', i);
      parts.push_back(p.substr(i, j == std::string::npos ? std::string::npos : j - i));
      if (j == std::string::npos) break;
      i = j;
    }
    return parts;
  }

  void reply_err(Reply* rep, const ApiErr& e) {
    rep->obj = Ref();
    rep->status = e.code;
    rep->body = status_body(e);
    rep->content_type = "application/json";
  }

  void reply_obj(Reply* rep, int status, const Ref& obj) {
    rep->status = status;
    rep->body.clear();
    rep->obj = obj;
  }

  // parse a request path to a resource route; false: not a resource path
  struct Route {
    Resource* ri = nullptr;
    std::string ns, name, sub, verb;
  };

  // 0: route found; 1: not a resource path (fallback); 2: error set
  int route(const Request& r, Route* rt, ApiErr* err) {
    const std::vector<std::string> parts = split_path(r.path);
    if (parts.empty()) return 1;
    std::string group, version;
    size_t rest;
    if (parts[0] == "api") {
      if (parts.size() < 3) return 1;
      version = parts[1];
      rest = 2;
    } else if (parts[0] == "apis") {
      if (parts.size() == 3) return 1;  // group-version discovery
      if (parts.size() < 4) return 1;
      group = parts[1];
      version = parts[2];
      rest = 3;
    } else {
      return 1;
    }
    if (parts[rest] == "namespaces" && parts.size() - rest >= 3) {
      rt->ns = parts[rest + 1];
      rest += 2;
    }
    const size_t left = parts.size() - rest;
    if (left > 3) {
      *err = mkerr(404, "NotFound", "the server could not find the requested resource");
      return 2;
    }
    const std::string& resource = parts[rest];
    if (left > 1) rt->name = parts[rest + 1];
    if (left > 2) rt->sub = parts[rest + 2];
    rt->ri = find(group, version, resource);
    if (!rt->ri) {
      *err = mkerr(404, "NotFound", group.empty() ? "the server could not find the requested resource (" +
                                                        resource + ")"
                                                  : "the server could not find the requested resource (" +
                                                        resource + "." + group + ")");
      return 2;
    }
    if (!rt->ri->namespaced && !rt->ns.empty()) {
      *err = mkerr(404, "NotFound", "the server could not find the requested resource");
      return 2;
    }
    const std::string& m = r.method;
    if (m == "GET") {
      const std::string w = r.qv("watch");
      rt->verb = !rt->name.empty() ? "get" : ((w == "true" || w == "1") ? "watch" : "list");
    } else if (m == "POST") {
      rt->verb = "create";
    } else if (m == "PUT") {
      rt->verb = "update";
    } else if (m == "PATCH") {
      rt->verb = "patch";
    } else if (m == "DELETE") {
      rt->verb = rt->name.empty() ? "deletecollection" : "delete";
    } else {
      *err = mkerr(405, "MethodNotAllowed", "method " + m + " not allowed");
      return 2;
    }
    return 0;
  }

  double delay_for(const std::string& verb, Resource* ri, const std::string& ns) {
    if (latency.empty()) return 0.0;
    auto it = latency.find(verb);
    double d = it != latency.end() ? it->second : 0.0;
    if (it == latency.end()) {
      auto st = latency.find("*");
      if (st != latency.end()) d = st->second;
    }
    if (verb == "list" && d > 0) {
      // a real apiserver scans the namespace for a label-selected LIST (harness.py LATENCY_PROFILES)
      auto po = latency.find("list_per_object");
      if (po != latency.end() && po->second > 0) {
        const std::string* nsp = (ri->namespaced && !ns.empty()) ? &ns : nullptr;
        d += po->second * static_cast<double>(count(ri, nsp));
      }
    }
    return d;
  }

  // the whole request (route, apply, serialise); the watch verb is started by the caller
  // returns false when the request is not ours (the Python fallback answers it)
  bool handle(const Request& r, Reply* rep, Route* rt_out, double* delay) {
    ++requests;
    if (discovery(r.path, rep)) return true;
    ApiErr err;
    Route rt;
    const int k = route(r, &rt, &err);
    if (k == 1) {
      const std::vector<std::string> parts = split_path(r.path);
      if (parts.size() == 3 && parts[0] == "apis") {  // /apis/<group>/<version>
        std::string o;
        bool any = false;
        for (Resource* rr : order)
          if (rr->group == parts[1] && rr->version == parts[2]) {
            if (any) o += ",";
            any = true;
            o += discovery_entry(rr);
          }
        if (!any) {
          reply_err(rep, mkerr(404, "NotFound", "the server could not find the requested resource"));
          return true;
        }
        rep->body = "{\"kind\":\"APIResourceList\",\"apiVersion\":\"v1\",\"groupVersion\":\"" + parts[1] + "/" +
                    parts[2] + "\",\"resources\":[" + o + "]}";
        return true;
      }
      return false;
    }
    if (k == 2) {
      reply_err(rep, err);
      return true;
    }
    // what the Python front end serves instead: server-side Table printing, JSON patch
    if ((rt.verb == "get" || rt.verb == "list") && r.accept.find("as=Table") != std::string::npos) return false;
    if (rt.verb == "patch" && r.content_type == "application/json-patch+json") return false;
    *rt_out = rt;
    if (delay) *delay = delay_for(rt.verb, rt.ri, rt.ns);
    return true;
  }

  // apply a routed request (after its injected latency)
  void apply(const Request& r, const Route& rt, Reply* rep) {
    ApiErr err;
    Resource* ri = rt.ri;
    const std::string& verb = rt.verb;
    if (verb == "list") {
      Selector sel;
      std::string serr;
      if (!sel.parse_labels(r.qv("labelSelector"), &serr) || !sel.parse_fields(r.qv("fieldSelector"), &serr)) {
        reply_err(rep, bad_request(serr));
        return;
      }
      const std::string lim = r.qv("limit");
      const long long limit = lim.empty() ? 0 : std::strtoll(lim.c_str(), nullptr, 10);
      rep->body.clear();
      if (!v_list(ri, rt.ns, sel, limit, r.qv("continue"), &rep->body, &err)) reply_err(rep, err);
      return;
    }
    if (verb == "get") {
      Ref o = v_get(ri, rt.ns, rt.name, &err);
      if (!o) reply_err(rep, err);
      else reply_obj(rep, 200, o);
      return;
    }
    Ref body;
    if (!r.body.empty()) {
      std::string perr;
      PhaseTimer pt(&phase[kParse]);
      body = jdom::parse(r.body.data(), r.body.size(), &perr);
      if (!body) {
        reply_err(rep, bad_request("invalid JSON body: " + perr));
        return;
      }
    }
    if (verb == "create" || verb == "update") {
      if (!body || !body->is_obj()) {
        reply_err(rep, bad_request("request body must be a JSON object"));
        return;
      }
    }
    Ref out;
    int status = 200;
    if (verb == "create") {
      out = v_create(ri, rt.ns, body, r.qv("dryRun") == "All", &err);
      status = 201;
    } else if (verb == "update") {
      out = v_update(ri, rt.ns, rt.name, body, rt.sub, &err);
    } else if (verb == "patch") {
      std::string ptype;
      if (r.content_type == "application/merge-patch+json") ptype = "merge";
      else if (r.content_type == "application/strategic-merge-patch+json") ptype = "strategic";
      if (ptype.empty()) {
        reply_err(rep, mkerr(415, "UnsupportedMediaType",
                             "the body of the request was in an unknown format - accepted media types include: "
                             "application/merge-patch+json, application/json-patch+json, "
                             "application/strategic-merge-patch+json"));
        return;
      }
      if (!body) {
        reply_err(rep, bad_request("merge patch must be a JSON object"));
        return;
      }
      out = v_patch(ri, rt.ns, rt.name, body, ptype, rt.sub, &err);
    } else if (verb == "delete") {
      std::string policy = r.qv("propagationPolicy");
      const Node* pre = nullptr;
      if (body && body->is_obj()) {
        if (!body->str("propagationPolicy").empty()) policy = body->str("propagationPolicy");
        pre = body->getn("preconditions");
      }
      out = v_delete(ri, rt.ns, rt.name, policy, pre, &err);
    } else if (verb == "deletecollection") {
      Selector sel;
      std::string serr;
      if (!sel.parse_labels(r.qv("labelSelector"), &serr)) {
        reply_err(rep, bad_request(serr));
        return;
      }
      std::vector<std::pair<std::string, std::string>> victims;
      for (auto& kv : ri->store->data)
        if (rt.ns.empty() || !ri->namespaced || kv.first == rt.ns)
          for (auto& ob : kv.second)
            if (sel.match(ob.second.get())) victims.emplace_back(kv.first, ob.first);
      record("list", ri);
      long long n = 0;
      for (auto& v : victims) {
        ApiErr e2;
        if (v_delete(ri, v.first, v.second, "", nullptr, &e2)) ++n;
      }
      rep->body = "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"status\":\"Success\",\"details\":{\"deleted\":" +
                  std::to_string(n) + "}}";
      return;
    }
    if (!out) {
      reply_err(rep, err);
      return;
    }
    reply_obj(rep, status, out);
  }

  // ---------------------------------------------------------------- watches
  // start a watch on connection c (or, c == nullptr, validate only); false + err on a bad request
  Watcher* start_watch(Conn* c, const Request& r, const Route& rt, ApiErr* err) {
    record("watch", rt.ri);
    auto w = std::make_unique<Watcher>();
    w->conn = c;
    w->res = rt.ri;
    w->ns = rt.ri->namespaced ? rt.ns : std::string();
    std::string serr;
    if (!w->sel.parse_labels(r.qv("labelSelector"), &serr) || !w->sel.parse_fields(r.qv("fieldSelector"), &serr)) {
      *err = bad_request(serr);
      return nullptr;
    }
    const std::string ab = r.qv("allowWatchBookmarks");
    w->bookmarks = ab == "true" || ab == "1";
    const std::string rvs = r.qv("resourceVersion");
    const std::string sie = r.qv("sendInitialEvents");
    Store* st = rt.ri->store;
    if (rvs.empty() || rvs == "0" || sie == "true") {
      for (auto& kv : st->data) {
        if (!w->ns.empty() && kv.first != w->ns) continue;
        for (auto& ob : kv.second)
          if (w->sel.match(ob.second.get())) put_event(w.get(), 0, ob.second.get());
      }
    } else {
      char* end = nullptr;
      const long long since = std::strtoll(rvs.c_str(), &end, 10);
      if (!end || *end) {
        *err = bad_request("invalid resourceVersion '" + rvs + "'");
        return nullptr;
      }
      if (since < st->floor) {
        *err = mkerr(410, "Expired", "too old resource version: " + std::to_string(since) + " (" +
                                         std::to_string(st->floor + 1) + ")");
        return nullptr;
      }
      // the log keeps each event's name, namespace and labels: a field selector on any other
      // field cannot be replayed, and the watcher relists (as past a compacted revision)
      for (const FieldReq& f : w->sel.fields)
        if (!(f.path.size() == 2 && f.path[0] == "metadata" && (f.path[1] == "name" || f.path[1] == "namespace"))) {
          *err = mkerr(410, "Expired", "too old resource version: " + std::to_string(since) + " (" +
                                           std::to_string(rv + 1) + ")");
          return nullptr;
        }
      for (const Event& ev : st->log)
        if (ev.rv > since) {
          const bool now_in = w->in_scope(scope_tree(ev.scope).get());
          const bool was_in = ev.type == 1 && ev.old_scope.set ? w->in_scope(scope_tree(ev.old_scope).get()) : false;
          offer(w.get(), ev.type, std::string_view(ev.bytes), ev.old_scope.set, now_in, was_in);
        }
    }
    Watcher* out = w.release();
    st->watchers.push_back(out);
    return out;
  }

  void bookmark(Watcher* w) {
    if (!w->bookmarks || w->ended) return;
    std::string& p = event_sink(w);
    p.append("{\"type\":\"BOOKMARK\",\"object\":{\"kind\":");
    jdom::put_string(&p, w->res->kind);
    p.append(",\"apiVersion\":");
    jdom::put_string(&p, w->res->api_version);
    p.append(",\"metadata\":{\"resourceVersion\":\"" + std::to_string(rv) + "\"}}}\n");
    if (!w->dirty) {
      w->dirty = true;
      dirty_watchers.push_back(w);
    }
  }

  void drop_watcher(Watcher* w) {
    auto& ws = w->res->store->watchers;
    ws.erase(std::remove(ws.begin(), ws.end(), w), ws.end());
    w->ended = true;
  }

  // delete a dropped watcher (no pointer to it may stay in the end-of-turn list)
  void free_watcher(Watcher* w) {
    dirty_watchers.erase(std::remove(dirty_watchers.begin(), dirty_watchers.end(), w), dirty_watchers.end());
    delete w;
  }

  // ---------------------------------------------------------------- event loop
  void arm(Conn* c, bool out) {
    struct epoll_event ev;
    ev.events = EPOLLIN | EPOLLRDHUP | (out ? EPOLLOUT : 0u);
    ev.data.u64 = c->id;
    epoll_ctl(epfd, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = out;
  }

  void mark_dirty(Conn* c) {
    dirty_conns.push_back(c);
  }

  void close_conn(Conn* c) {
    if (c->closed) return;
    c->closed = true;
    if (c->watch) {
      drop_watcher(c->watch);
      free_watcher(c->watch);
      c->watch = nullptr;
    }
    epoll_ctl(epfd, EPOLL_CTL_DEL, c->fd, nullptr);
    if (c->ssl) {
      SSL_free(c->ssl);
      c->ssl = nullptr;
    }
    ::close(c->fd);
    c->fd = -1;
  }

  // write what is buffered; false: the connection failed (closed)
  bool flush(Conn* c) {
    if (c->closed) return false;
    if (c->watch && c->watch->chunk_at != std::string::npos) frame_pending(c->watch);
    while (c->out_off < c->out.size()) {
      const char* p = c->out.data() + c->out_off;
      const size_t n = c->out.size() - c->out_off;
      if (c->ssl) {
        const int w = SSL_write(c->ssl, p, static_cast<int>(std::min<size_t>(n, 1 << 30)));
        if (w <= 0) {
          const int e = SSL_get_error(c->ssl, w);
          if (e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_WANT_READ) {
            if (!c->want_out) arm(c, true);
            return true;
          }
          close_conn(c);
          return false;
        }
        c->out_off += static_cast<size_t>(w);
      } else {
        ++sends;
        const ssize_t w = ::send(c->fd, p, n, MSG_NOSIGNAL);
        if (w < 0) {
          if (errno == EAGAIN || errno == EWOULDBLOCK) {
            if (!c->want_out) arm(c, true);
            return true;
          }
          if (errno == EINTR) continue;
          close_conn(c);
          return false;
        }
        c->out_off += static_cast<size_t>(w);
      }
    }
    c->out.clear();
    c->out_off = 0;
    if (c->want_out) arm(c, false);
    if (c->close_after) {
      close_conn(c);
      return false;
    }
    return true;
  }

  static const char* reason(int s) {
    switch (s) {
      case 200: return "OK";
      case 201: return "Created";
      case 202: return "Accepted";
      case 204: return "No Content";
      case 400: return "Bad Request";
      case 401: return "Unauthorized";
      case 403: return "Forbidden";
      case 404: return "Not Found";
      case 405: return "Method Not Allowed";
      case 409: return "Conflict";
      case 410: return "Gone";
      case 413: return "Payload Too Large";
      case 415: return "Unsupported Media Type";
      case 422: return "Unprocessable Entity";
      case 429: return "Too Many Requests";
      case 431: return "Request Header Fields Too Large";
      case 500: return "Internal Server Error";
      case 501: return "Not Implemented";
      case 503: return "Service Unavailable";
      case 504: return "Gateway Timeout";
      default: return "Unknown";
    }
  }

  void write_reply(Conn* c, const Reply& rep, bool keep) {
    PhaseTimer pt(&phase[kReply]);
    const std::string_view body = rep.obj ? std::string_view(jdom::encoded(rep.obj.get())) : std::string_view(rep.body);
    std::string& o = c->out;
    o.append("HTTP/1.1 ");
    o.append(std::to_string(rep.status));
    o.push_back(' ');
    o.append(reason(rep.status));
    o.append("\r\nContent-Type: ");
    o.append(rep.content_type);
    o.append("\r\nContent-Length: ");
    o.append(std::to_string(body.size()));
    o.append("\r\n");
    o.append(rep.extra_headers);
    if (!keep) o.append("Connection: close\r\n");
    o.append("\r\n");
    o.append(body);
    if (!keep) c->close_after = true;
    mark_dirty(c);
  }

  void write_raw_error(Conn* c, int status, const char* msg) {
    Reply rep;
    rep.status = status;
    rep.body = msg;
    rep.content_type = "text/plain";
    write_reply(c, rep, false);
  }

  // the Python fallback (GIL taken); false: no fallback
  bool call_fallback(const Request& r, Reply* rep);

  void push_timer(double due, int kind, uint64_t conn_id) {
    timers.push(Timer{due, ++timer_seq, kind, conn_id});
  }

  // run one request on connection c (after parsing, or when its injected latency elapsed)
  void run_request(Conn* c, Request& r, bool delayed_done) {
    const unsigned long long t0 = __rdtsc();
    run_request_(c, r, delayed_done);
    cyc_verbs += __rdtsc() - t0;
  }

  void run_request_(Conn* c, Request& r, bool delayed_done) {
    Reply rep;
    Route rt;
    double delay = 0.0;
    if (!handle(r, &rep, &rt, delayed_done ? nullptr : &delay)) {
      const unsigned long long f0 = __rdtsc();
      if (!call_fallback(r, &rep)) reply_err(&rep, mkerr(404, "NotFound", "the server could not find the "
                                                                          "requested resource"));
      const unsigned long long f = __rdtsc() - f0;
      cyc_fallback += f;
      cyc_verbs -= f;  // counted once, as fallback
      write_reply(c, rep, r.keep);
      return;
    }
    if (!rt.ri) {  // discovery / errors
      write_reply(c, rep, r.keep);
      return;
    }
    if (!delayed_done && delay > 0) {
      c->busy = true;
      c->delayed = std::make_unique<Request>(std::move(r));
      push_timer(mono() + delay, 0, c->id);
      return;
    }
    if (rt.verb == "watch") {
      ApiErr err;
      Watcher* w = start_watch(c, r, rt, &err);
      if (!w) {
        reply_err(&rep, err);
        write_reply(c, rep, r.keep);
        return;
      }
      c->busy = true;
      c->watch = w;
      c->watch_keep = r.keep;
      c->out.append("HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n");
      frame_pending(w);  // the initial replay
      w->streaming = true;
      mark_dirty(c);
      const std::string ts = r.qv("timeoutSeconds");
      const double timeout = ts.empty() ? 1800.0 : std::strtod(ts.c_str(), nullptr);
      push_timer(mono() + (timeout > 0 ? timeout : 1800.0), 1, c->id);
      return;
    }
    const unsigned long long a0 = __rdtsc();
    apply(r, rt, &rep);
    write_reply(c, rep, r.keep);
    const unsigned long long a = __rdtsc() - a0;
    if (last_vk && last_vk->first.ri == rt.ri && last_vk->first.verb == rt.verb && last_vk->first.sub == rt.sub) {
      last_vk->second.first += a;
      ++last_vk->second.second;
    } else {
      auto it = verb_cpu.find(VerbKey{rt.ri, rt.verb, rt.sub});
      if (it == verb_cpu.end()) it = verb_cpu.emplace(VerbKey{rt.ri, rt.verb, rt.sub}, std::make_pair(0ULL, 0LL)).first;
      it->second.first += a;
      ++it->second.second;
      last_vk = &*it;
    }
  }
  void end_watch(Conn* c) {
    Watcher* w = c->watch;
    if (!w) return;
    frame_pending(w);
    drop_watcher(w);
    free_watcher(w);
    c->watch = nullptr;
    c->out.append("0\r\n\r\n");
    const bool keep = c->watch_keep;
    c->busy = false;
    if (!keep) c->close_after = true;
    mark_dirty(c);
    if (keep) drain(c);
  }

  void frame_pending(Watcher* w) {
    w->dirty = false;
    Conn* c = w->conn;
    if (!c || c->closed) {
      w->pending.clear();
      w->chunk_at = std::string::npos;
      return;
    }
    if (w->chunk_at != std::string::npos) {  // close the open chunk: fill in its size
      const size_t body = c->out.size() - w->chunk_at - 10;
      char hex[9];
      snprintf(hex, sizeof hex, "%08zx", body);
      std::memcpy(&c->out[w->chunk_at], hex, 8);
      c->out.append("\r\n");
      w->chunk_at = std::string::npos;
      mark_dirty(c);
    }
    if (w->pending.empty()) return;
    char hex[24];
    snprintf(hex, sizeof hex, "%zx\r\n", w->pending.size());
    c->out.append(hex);
    c->out.append(w->pending);
    c->out.append("\r\n");
    w->pending.clear();
    mark_dirty(c);
  }

  // parse and run buffered requests until the connection is busy or needs more bytes
  void drain(Conn* c) {
    while (!c->busy && !c->closed && !c->close_after) {
      Request r;
      const int st = parse_request(c, &r);
      if (st == 0) return;
      if (st < 0) return;  // error reply written
      run_request(c, r, false);
    }
  }

  // 1: a request; 0: need more bytes; -1: error (replied)
  static std::string_view sv_strip(std::string_view v) {
    size_t b = 0, e = v.size();
    while (b < e && (v[b] == ' ' || v[b] == '\t')) ++b;
    while (e > b && (v[e - 1] == ' ' || v[e - 1] == '\t')) --e;
    return v.substr(b, e - b);
  }
  static bool ieq(std::string_view a, const char* lit) {
    const size_t n = std::strlen(lit);
    if (a.size() != n) return false;
    for (size_t i = 0; i < n; ++i)
      if (std::tolower(static_cast<unsigned char>(a[i])) != lit[i]) return false;
    return true;
  }
  static std::string lower(std::string_view v) {
    std::string o(v);
    for (auto& ch : o) ch = static_cast<char>(std::tolower(static_cast<unsigned char>(ch)));
    return o;
  }

  // 1: a request; 0: need more bytes; -1: error (replied).  Header fields are read in place;
  // only the few the server uses are copied (the raw block is kept for the Python fallback).
  int parse_request(Conn* c, Request* r) {
    std::string& b = c->in;
    const size_t hend = b.find("\r\n\r\n");
    if (hend == std::string::npos) {
      if (b.size() > (1u << 20)) {
        write_raw_error(c, 431, "request header too large");
        return -1;
      }
      return 0;
    }
    const std::string_view all(b.data(), hend + 2);
    const size_t l_end = all.find("\r\n");
    const std::string_view line = all.substr(0, l_end);
    const size_t sp1 = line.find(' ');
    const size_t sp2 = sp1 == std::string_view::npos ? std::string_view::npos : line.find(' ', sp1 + 1);
    if (sp1 == std::string_view::npos || sp2 == std::string_view::npos) {
      write_raw_error(c, 400, "bad request line");
      return -1;
    }
    r->method.assign(line.data(), sp1);
    for (auto& ch : r->method) ch = static_cast<char>(std::toupper(static_cast<unsigned char>(ch)));
    std::string target(line.substr(sp1 + 1, sp2 - sp1 - 1));
    const std::string_view version = line.substr(sp2 + 1);
    long long clen = 0;
    bool chunked = false, expect = false, conn_close = false, conn_keep = false;
    size_t p = l_end + 2;
    r->raw_headers.assign(all.data() + p, all.size() > p ? all.size() - p : 0);
    while (p < all.size()) {
      const size_t nl = all.find("\r\n", p);
      if (nl == std::string_view::npos) break;
      const std::string_view ln = all.substr(p, nl - p);
      p = nl + 2;
      const size_t colon = ln.find(':');
      if (colon == std::string_view::npos) continue;
      const std::string_view k = sv_strip(ln.substr(0, colon));
      const std::string_view v = sv_strip(ln.substr(colon + 1));
      switch (k.size()) {
        case 14:  // content-length
          if (ieq(k, "content-length")) {
            std::string num(v);
            char* e = nullptr;
            clen = std::strtoll(num.c_str(), &e, 10);
            if (num.empty() || !e || *e || clen < 0) {
              write_raw_error(c, 400, "bad request");
              return -1;
            }
          }
          break;
        case 17:  // transfer-encoding
          if (ieq(k, "transfer-encoding")) chunked = lower(v).find("chunked") != std::string::npos;
          break;
        case 12:  // content-type
          if (ieq(k, "content-type")) r->content_type = lower(sv_strip(v.substr(0, v.find(';'))));
          break;
        case 6:  // accept, expect
          if (ieq(k, "accept")) r->accept.assign(v);
          else if (ieq(k, "expect")) expect = ieq(v, "100-continue");
          break;
        case 10:  // connection
          if (ieq(k, "connection")) {
            conn_close = ieq(v, "close");
            conn_keep = ieq(v, "keep-alive");
          }
          break;
        case 13:  // authorization
          if (ieq(k, "authorization")) r->authorization.assign(v);
          break;
        default: break;
      }
    }
    size_t pos = hend + 4;
    if (chunked) {
      std::string body;
      while (true) {
        const size_t nl = b.find("\r\n", pos);
        if (nl == std::string::npos) return 0;
        long long size = 0;
        std::string sz = b.substr(pos, nl - pos);
        sz = sz.substr(0, sz.find(';'));
        char* e = nullptr;
        size = std::strtoll(Selector::strip(sz).c_str(), &e, 16);
        if (!e || *e || size < 0) {
          write_raw_error(c, 400, "bad request");
          return -1;
        }
        if (size == 0) {
          const size_t tend = b.find("\r\n\r\n", nl);
          if (tend == std::string::npos) return 0;
          pos = tend + 4;
          break;
        }
        if (b.size() < nl + 2 + static_cast<size_t>(size) + 2) return 0;
        body.append(b, nl + 2, static_cast<size_t>(size));
        pos = nl + 2 + static_cast<size_t>(size) + 2;
      }
      r->body = std::move(body);
    } else {
      if (clen > (64LL << 20)) {
        write_raw_error(c, 413, "request body too large");
        return -1;
      }
      if (b.size() < pos + static_cast<size_t>(clen)) {
        if (expect && !c->continued) {
          c->continued = true;
          c->out.append("HTTP/1.1 100 Continue\r\n\r\n");
          mark_dirty(c);
        }
        return 0;
      }
      r->body.assign(b, pos, static_cast<size_t>(clen));
      pos += static_cast<size_t>(clen);
    }
    b.erase(0, pos);
    c->continued = false;
    r->keep = version == "HTTP/1.1" ? !conn_close : conn_keep;
    // absolute form (a client behind a proxy): routing needs the path and query only
    const size_t scheme = target.find("://");
    if (!target.empty() && target[0] != '/' && scheme != std::string::npos) {
      const size_t slash = target.find('/', scheme + 3);
      const size_t qm = target.find('?', scheme + 3);
      if (slash == std::string::npos || (qm != std::string::npos && qm < slash))
        target = "/" + (qm != std::string::npos ? target.substr(qm) : std::string());
      else
        target = target.substr(slash);
    }
    const size_t qm = target.find('?');
    std::string path = target.substr(0, qm);
    if (path.find('%') != std::string::npos) path = url_decode(path, false);
    r->path = std::move(path);
    if (qm != std::string::npos) {
      r->query_string = target.substr(qm + 1);
      parse_query(r->query_string, &r->query);
    }
    return 1;
  }

  void accept_all() {
    while (true) {
      sockaddr_storage sa;
      socklen_t sl = sizeof sa;
      const int fd = ::accept4(lfd, reinterpret_cast<sockaddr*>(&sa), &sl, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (fd < 0) return;
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
      Conn* c = new Conn();
      c->fd = fd;
      c->id = next_conn_id++;
      if (ssl_ctx) {
        c->ssl = SSL_new(ssl_ctx);
        SSL_set_fd(c->ssl, fd);
        SSL_set_accept_state(c->ssl);
        c->handshaking = true;
      }
      conns[c->id] = c;
      struct epoll_event ev;
      ev.events = EPOLLIN | EPOLLRDHUP;
      ev.data.u64 = c->id;
      epoll_ctl(epfd, EPOLL_CTL_ADD, fd, &ev);
    }
  }

  void on_readable(Conn* c) {
    const unsigned long long t0 = __rdtsc();
    const unsigned long long v0 = cyc_verbs + cyc_fallback;
    on_readable_(c);
    // reading and parsing: what the verbs run from here did not take
    cyc_read += __rdtsc() - t0 - (cyc_verbs + cyc_fallback - v0);
  }

  void on_readable_(Conn* c) {
    char buf[65536];
    bool eof = false;
    if (c->ssl) {
      if (c->handshaking) {
        const int r = SSL_do_handshake(c->ssl);
        if (r != 1) {
          const int e = SSL_get_error(c->ssl, r);
          if (e == SSL_ERROR_WANT_READ) return;
          if (e == SSL_ERROR_WANT_WRITE) {
            arm(c, true);
            return;
          }
          close_conn(c);
          return;
        }
        c->handshaking = false;
      }
      while (true) {
        const int n = SSL_read(c->ssl, buf, sizeof buf);
        if (n > 0) {
          c->in.append(buf, static_cast<size_t>(n));
          continue;
        }
        const int e = SSL_get_error(c->ssl, n);
        if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) break;
        eof = true;
        break;
      }
    } else {
      while (true) {
        const ssize_t n = ::recv(c->fd, buf, sizeof buf, 0);
        if (n > 0) {
          c->in.append(buf, static_cast<size_t>(n));
          if (static_cast<size_t>(n) < sizeof buf) break;
          continue;
        }
        if (n == 0) {
          eof = true;
          break;
        }
        if (errno == EINTR) continue;
        if (errno != EAGAIN && errno != EWOULDBLOCK) eof = true;
        break;
      }
    }
    if (!c->busy) drain(c);
    if (eof && !c->closed) {
      // the peer is gone: what it sent is answered (best effort) and the connection closed
      flush(c);
      close_conn(c);
    }
  }

  void on_writable(Conn* c) {
    if (c->ssl && c->handshaking) {
      on_readable(c);
      return;
    }
    flush(c);
  }

  void run_timers() {
    const double now = mono();
    while (!timers.empty() && timers.top().due <= now) {
      const Timer t = timers.top();
      timers.pop();
      if (t.kind == 2) {
        for (auto& kv : stores)
          for (Watcher* w : kv.second->watchers) bookmark(w);
        push_timer(now + bookmark_interval, 2, 0);
        continue;
      }
      auto it = conns.find(t.conn_id);
      if (it == conns.end() || it->second->closed) continue;
      Conn* c = it->second;
      if (t.kind == 0) {
        if (!c->delayed) continue;
        std::unique_ptr<Request> r = std::move(c->delayed);
        c->busy = false;
        run_request(c, *r, true);
        if (!c->busy) drain(c);
      } else if (t.kind == 1) {
        if (c->watch) end_watch(c);
      }
    }
  }

  void end_of_turn(bool flush_watches = true) {
    const unsigned long long t0 = __rdtsc();
    end_of_turn_(flush_watches);
    cyc_write += __rdtsc() - t0;
  }

  static bool streaming_watch(const Conn* c) { return c->watch && c->watch->streaming && !c->close_after; }

  void end_of_turn_(bool flush_watches) {
    // a streaming watch's events may wait for a quiet turn; everything else goes out now
    bool deferred = false;
    std::vector<Watcher*> ws;
    ws.swap(dirty_watchers);
    for (Watcher* w : ws) {
      if (!w->dirty) continue;
      if (!flush_watches && w->conn && !w->conn->closed && streaming_watch(w->conn)) {
        dirty_watchers.push_back(w);
        deferred = true;
        continue;
      }
      frame_pending(w);
    }
    // flush each dirty connection once
    std::vector<Conn*> cs;
    cs.swap(dirty_conns);
    std::unordered_set<Conn*> seen;
    for (Conn* c : cs) {
      if (!seen.insert(c).second) continue;
      if (c->closed) continue;
      if (!flush_watches && streaming_watch(c)) {
        dirty_conns.push_back(c);
        deferred = true;
        continue;
      }
      flush(c);  // frames the watch's open chunk first
    }
    if (deferred && !watch_deferred) watch_defer_since = mono();
    watch_deferred = deferred;
    // reap closed connections (none may stay deferred)
    if (!dirty_conns.empty())
      dirty_conns.erase(std::remove_if(dirty_conns.begin(), dirty_conns.end(), [](Conn* c) { return c->closed; }),
                        dirty_conns.end());
    for (auto it = conns.begin(); it != conns.end();) {
      if (it->second->closed) {
        delete it->second;
        it = conns.erase(it);
      } else {
        ++it;
      }
    }
  }

  // one turn's share of the queued completion writes (accounted with the fallback's controls)
  void run_pending_patches() {
    const unsigned long long t0 = __rdtsc();
    PendingPatches& p = pending_patches.front();
    Resource* ri = find(p.g, p.v, p.r);
    if (!ri) p.next = p.todo.size();
    for (size_t k = 0; k < p.per_turn && p.next < p.todo.size(); ++k) {
      const auto& t = p.todo[p.next++];
      Ref patch = subst(p.tree, p.ph, t.second);
      ApiErr err;
      if (v_patch(ri, t.first, t.second, patch, "merge", p.sub, &err)) ++pending_applied;
    }
    if (p.next >= p.todo.size()) pending_patches.pop_front();
    cyc_fallback += __rdtsc() - t0;
  }

  void loop() {
    loop_tid.store(static_cast<pid_t>(syscall(SYS_gettid)));
    if (const char* e = std::getenv("APISERVERD_WATCH_DEFER_S")) watch_defer_s = std::strtod(e, nullptr);
    if (const char* e = std::getenv("APISERVERD_LOG_TREES")) log_trees = e[0] == '1';
    std::vector<struct epoll_event> evs(256);
    push_timer(mono() + bookmark_interval, 2, 0);
    while (!stopping.load()) {
      int timeout_ms = 1000;
      if (!timers.empty()) {
        const double d = timers.top().due - mono();
        timeout_ms = d <= 0 ? 0 : static_cast<int>(std::min(1000.0, std::ceil(d * 1000.0)));
      }
      // poll: the deferred watch events go out once idle; queued completion writes continue
      if (watch_deferred || !pending_patches.empty()) timeout_ms = 0;
      const int n = epoll_wait(epfd, evs.data(), static_cast<int>(evs.size()), timeout_ms);
      std::lock_guard<std::recursive_mutex> g(mu);
      const long long turn0 = thread_cpu_ns();
      const unsigned long long tc0 = __rdtsc();
      for (int i = 0; i < n; ++i) {
        const uint64_t id = evs[i].data.u64;
        if (id == UINT64_MAX - 1) {
          accept_all();
          continue;
        }
        if (id == UINT64_MAX) {
          uint64_t v;
          (void)!::read(evfd, &v, sizeof v);
          continue;
        }
        auto it = conns.find(id);
        if (it == conns.end() || it->second->closed) continue;
        Conn* c = it->second;
        const uint32_t e = evs[i].events;
        if (e & EPOLLOUT) on_writable(c);
        if (!c->closed && (e & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR))) on_readable(c);
      }
      run_timers();
      if (!pending_patches.empty()) run_pending_patches();
      ++turns;
      end_of_turn(n == 0 || watch_defer_s <= 0.0 || (watch_deferred && mono() - watch_defer_since >= watch_defer_s));
      cyc_loop += __rdtsc() - tc0;
      cpu_loop += thread_cpu_ns() - turn0;
    }
    // shutdown: end every watch and close every connection
    std::lock_guard<std::recursive_mutex> g(mu);
    for (auto& kv : conns) {
      Conn* c = kv.second;
      if (c->watch) {
        drop_watcher(c->watch);
        free_watcher(c->watch);
        c->watch = nullptr;
      }
      if (!c->closed) close_conn(c);
    }
    end_of_turn();
  }

  // ---------------------------------------------------------------- start / stop
  bool start(const std::string& host, int port_in, const std::string& cert, const std::string& key, std::string* err) {
    if (!cert.empty()) {
      ssl_ctx = SSL_CTX_new(TLS_server_method());
      if (!ssl_ctx || SSL_CTX_use_certificate_chain_file(ssl_ctx, cert.c_str()) != 1 ||
          SSL_CTX_use_PrivateKey_file(ssl_ctx, key.c_str(), SSL_FILETYPE_PEM) != 1) {
        *err = "TLS setup failed (certificate or key)";
        return false;
      }
      SSL_CTX_set_mode(ssl_ctx, SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER | SSL_MODE_ENABLE_PARTIAL_WRITE);
    }
    lfd = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    int one = 1;
    setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons(static_cast<uint16_t>(port_in));
    if (inet_pton(AF_INET, host.c_str(), &sa.sin_addr) != 1) {
      *err = "bad host address " + host;
      return false;
    }
    if (::bind(lfd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 || ::listen(lfd, 1024) != 0) {
      *err = std::string("bind/listen failed: ") + strerror(errno);
      return false;
    }
    socklen_t sl = sizeof sa;
    getsockname(lfd, reinterpret_cast<sockaddr*>(&sa), &sl);
    port = ntohs(sa.sin_port);
    epfd = epoll_create1(EPOLL_CLOEXEC);
    evfd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    struct epoll_event ev;
    ev.events = EPOLLIN;
    ev.data.u64 = UINT64_MAX - 1;
    epoll_ctl(epfd, EPOLL_CTL_ADD, lfd, &ev);
    ev.data.u64 = UINT64_MAX;
    epoll_ctl(epfd, EPOLL_CTL_ADD, evfd, &ev);
    running = true;
    thread = std::thread([this] { loop(); });
    return true;
  }

  // make the loop's epoll_wait return (work queued from another thread)
  void wake() {
    const uint64_t one = 1;
    (void)!::write(evfd, &one, sizeof one);
  }

  void stop() {
    if (!running) return;
    stopping.store(true);
    const uint64_t one = 1;
    (void)!::write(evfd, &one, sizeof one);
    thread.join();
    running = false;
    ::close(lfd);
    ::close(epfd);
    ::close(evfd);
    lfd = epfd = evfd = -1;
  }
};

#ifdef APISERVERD_STANDALONE
bool Impl::call_fallback(const Request&, Reply*) { return false; }
}  // namespace
#else
// the Python fallback: fallback(method, path, query_string, headers, body) -> (status, body, ctype) | None
bool Impl::call_fallback(const Request& r, Reply* rep) {
  if (!fallback) return false;
  PyGILState_STATE g = PyGILState_Ensure();
  bool ok = false;
  PyObject* hdrs = PyDict_New();  // lower-cased names
  {
    const std::string_view all(r.raw_headers);
    size_t p = 0;
    while (p < all.size()) {
      size_t nl = all.find("\r\n", p);
      if (nl == std::string_view::npos) nl = all.size();
      const std::string_view ln = all.substr(p, nl - p);
      p = nl + 2;
      const size_t colon = ln.find(':');
      if (colon == std::string_view::npos) continue;
      const std::string k = Impl::lower(Impl::sv_strip(ln.substr(0, colon)));
      const std::string_view v = Impl::sv_strip(ln.substr(colon + 1));
      PyObject* pv = PyUnicode_DecodeLatin1(v.data(), static_cast<Py_ssize_t>(v.size()), nullptr);
      if (pv) {
        PyDict_SetItemString(hdrs, k.c_str(), pv);
        Py_DECREF(pv);
      }
    }
  }
  PyObject* res = PyObject_CallFunction(fallback, "ssNNy#", r.method.c_str(), r.path.c_str(),
                                        PyUnicode_DecodeLatin1(r.query_string.data(),
                                                               static_cast<Py_ssize_t>(r.query_string.size()),
                                                               nullptr),
                                        hdrs, r.body.data(), static_cast<Py_ssize_t>(r.body.size()));
  if (!res) {
    PyErr_Print();
    rep->status = 500;
    rep->body = status_body(mkerr(500, "InternalError", "fallback handler failed"));
    ok = true;
  } else if (res == Py_None) {
    ok = false;
  } else {
    int status = 200;
    const char* b = nullptr;
    Py_ssize_t bl = 0;
    const char* ct = "application/json";
    PyObject* extra = nullptr;
    if (PyArg_ParseTuple(res, "iy#|sO", &status, &b, &bl, &ct, &extra)) {
      rep->status = status;
      rep->body.assign(b, static_cast<size_t>(bl));
      rep->content_type = ct;
      if (extra && PyDict_Check(extra)) {
        PyObject *k, *v;
        Py_ssize_t pos = 0;
        while (PyDict_Next(extra, &pos, &k, &v)) {
          const char* ks = PyUnicode_AsUTF8(k);
          const char* vs = PyUnicode_AsUTF8(v);
          if (ks && vs) rep->extra_headers += std::string(ks) + ": " + vs + "\r\n";
        }
      }
      ok = true;
    } else {
      PyErr_Print();
      rep->status = 500;
      rep->body = status_body(mkerr(500, "InternalError", "fallback returned a bad value"));
      ok = true;
    }
    Py_DECREF(res);
  }
  PyGILState_Release(g);
  return ok;
}

// ====================================================================== Python binding

PyObject* Server_new(PyTypeObject* type, PyObject*, PyObject*) {
  Server* self = reinterpret_cast<Server*>(type->tp_alloc(type, 0));
  if (self) self->impl = new Impl();
  return reinterpret_cast<PyObject*>(self);
}

int Server_init(Server* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"now_ns", "watch_window", "bookmark_interval", nullptr};
  long long now = 0;
  Py_ssize_t window = 200000;
  double bm = 60.0;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "|Lnd", const_cast<char**>(kwlist), &now, &window, &bm)) return -1;
  Impl* s = self->impl;
  // The server thread allocates from a secondary malloc arena, which glibc grows (mprotect) and
  // trims back (madvise) around a small top chunk: with trees retired by the thousand per tick
  // it thrashed -- the stack sampler put __default_morecore + mprotect + the page faults behind
  // them at a fifth of the server's CPU.  This process only serves: keep what it has.
  mallopt(M_TRIM_THRESHOLD, 1 << 30);
  mallopt(M_TOP_PAD, 64 << 20);
  mallopt(M_MMAP_THRESHOLD, 64 << 20);
  s->now_ns = now;
  s->watch_window = static_cast<size_t>(std::max<Py_ssize_t>(1, window));
  s->bookmark_interval = bm > 0 ? bm : 1e9;
  if (s->resources.empty()) s->builtins();
  return 0;
}

void Server_dealloc(Server* self) {
  if (self->impl) {
    Py_BEGIN_ALLOW_THREADS
    self->impl->stop();
    Py_END_ALLOW_THREADS
    Py_XDECREF(self->impl->fallback);
    delete self->impl;
    self->impl = nullptr;
  }
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// request(method, path, query="", body=b"", content_type="") -> (status, body bytes)
PyObject* Server_request(Server* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"method", "path", "query", "body", "content_type", "accept", nullptr};
  const char *m, *p, *q = "", *ct = "", *acc = "";
  const char* b = "";
  Py_ssize_t bl = 0, ql = 0;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "ss|s#y#ss", const_cast<char**>(kwlist), &m, &p, &q, &ql, &b, &bl, &ct,
                                   &acc))
    return nullptr;
  Request r;
  r.method = m;
  r.path = p;
  r.content_type = ct;
  r.accept = acc;
  r.body.assign(b, static_cast<size_t>(bl));
  r.query_string.assign(q, static_cast<size_t>(ql));
  parse_query(r.query_string, &r.query);
  Reply rep;
  bool handled;
  Impl* s = self->impl;
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    Impl::Route rt;
    handled = s->handle(r, &rep, &rt, nullptr);
    if (handled && rt.ri) {
      if (rt.verb == "watch") {
        rep.status = 400;
        rep.body = status_body(bad_request("watch is served over HTTP only"));
      } else {
        s->apply(r, rt, &rep);
      }
    }
    // events of this write reach the watchers now -- unless this runs on the server thread (a
    // fallback handler's call): its loop ends the turn, and must not find connections reaped
    if (!s->running || std::this_thread::get_id() != s->thread.get_id()) s->end_of_turn();
  }
  Py_END_ALLOW_THREADS
  if (!handled) return Py_BuildValue("(iy)", 404, "");
  const std::string_view body = rep.obj ? std::string_view(jdom::encoded(rep.obj.get())) : std::string_view(rep.body);
  return Py_BuildValue("(iy#)", rep.status, body.data(), static_cast<Py_ssize_t>(body.size()));
}

PyObject* Server_start(Server* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"host", "port", "certfile", "keyfile", nullptr};
  const char* host = "127.0.0.1";
  int port = 0;
  const char *cert = "", *key = "";
  if (!PyArg_ParseTupleAndKeywords(args, kw, "|siss", const_cast<char**>(kwlist), &host, &port, &cert, &key))
    return nullptr;
  std::string err;
  bool ok;
  Py_BEGIN_ALLOW_THREADS
  ok = self->impl->start(host, port, cert, key, &err);
  Py_END_ALLOW_THREADS
  if (!ok) {
    PyErr_SetString(PyExc_OSError, err.c_str());
    return nullptr;
  }
  return PyLong_FromLong(self->impl->port);
}

PyObject* Server_stop(Server* self, PyObject*) {
  Py_BEGIN_ALLOW_THREADS
  self->impl->stop();
  Py_END_ALLOW_THREADS
  Py_RETURN_NONE;
}

PyObject* Server_set_clock(Server* self, PyObject* arg) {
  const long long v = PyLong_AsLongLong(arg);
  if (v == -1 && PyErr_Occurred()) return nullptr;
  Impl* s = self->impl;
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    s->now_ns = v;
  }
  Py_END_ALLOW_THREADS
  Py_RETURN_NONE;
}

PyObject* Server_now_ns(Server* self, PyObject*) { return PyLong_FromLongLong(self->impl->now_ns); }

PyObject* Server_set_latency(Server* self, PyObject* arg) {
  if (!PyDict_Check(arg)) {
    PyErr_SetString(PyExc_TypeError, "set_latency(dict of verb -> seconds)");
    return nullptr;
  }
  std::map<std::string, double> lat;
  PyObject *k, *v;
  Py_ssize_t pos = 0;
  while (PyDict_Next(arg, &pos, &k, &v)) {
    const char* ks = PyUnicode_AsUTF8(k);
    const double d = PyFloat_AsDouble(v);
    if (!ks || (d == -1.0 && PyErr_Occurred())) return nullptr;
    lat[ks] = d;
  }
  Impl* s = self->impl;
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    for (auto& kv : lat) s->latency[kv.first] = kv.second;
  }
  Py_END_ALLOW_THREADS
  Py_RETURN_NONE;
}

PyObject* Server_clear_latency(Server* self, PyObject*) {
  Impl* s = self->impl;
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    s->latency.clear();
  }
  Py_END_ALLOW_THREADS
  Py_RETURN_NONE;
}

PyObject* Server_set_fallback(Server* self, PyObject* arg) {
  PyObject* old = self->impl->fallback;
  if (arg == Py_None) {
    self->impl->fallback = nullptr;
  } else {
    Py_INCREF(arg);
    self->impl->fallback = arg;
  }
  Py_XDECREF(old);
  Py_RETURN_NONE;
}

PyObject* Server_stats(Server* self, PyObject*) {
  Impl* s = self->impl;
  std::map<std::string, long long> bv, brv;
  std::map<std::string, std::pair<long long, long long>> vcpu;
  unsigned long long ph[Impl::kPhases];
  long long total, rv, reqs;
  long long cpu[6];
  long long io[2];
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    for (auto& kv : s->rec_counts) {
      bv[kv.first.second] += kv.second;
      brv[kv.first.first->resource + ":" + kv.first.second] += kv.second;
    }
    total = s->stats_total;
    rv = s->rv;
    reqs = s->requests;
    // cycles -> thread CPU ns, at the ratio the turns ran at
    const double ns_per_cyc = s->cyc_loop ? static_cast<double>(s->cpu_loop) / static_cast<double>(s->cyc_loop) : 0.0;
    cpu[0] = static_cast<long long>(static_cast<double>(s->cyc_read) * ns_per_cyc);
    cpu[1] = static_cast<long long>(static_cast<double>(s->cyc_verbs) * ns_per_cyc);
    cpu[2] = static_cast<long long>(static_cast<double>(s->cyc_fallback) * ns_per_cyc);
    cpu[3] = static_cast<long long>(static_cast<double>(s->cyc_write) * ns_per_cyc);
    cpu[4] = s->cpu_loop;
    cpu[5] = s->slow_admits;
    io[0] = s->sends;
    io[1] = s->turns;
    for (auto& kv : s->verb_cpu) {
      const std::string key = kv.first.verb + (kv.first.sub.empty() ? "" : "/" + kv.first.sub) + ":" +
                              kv.first.ri->resource;
      auto& e = vcpu[key];
      e.first += static_cast<long long>(static_cast<double>(kv.second.first) * ns_per_cyc);
      e.second += kv.second.second;
    }
    for (int i = 0; i < Impl::kPhases; ++i) ph[i] = s->phase[i];
  }
  Py_END_ALLOW_THREADS
  PyObject* d = PyDict_New();
  PyObject* a = PyDict_New();
  for (auto& kv : bv) {
    PyObject* v = PyLong_FromLongLong(kv.second);
    PyDict_SetItemString(a, kv.first.c_str(), v);
    Py_DECREF(v);
  }
  PyObject* b = PyDict_New();
  for (auto& kv : brv) {
    PyObject* v = PyLong_FromLongLong(kv.second);
    PyDict_SetItemString(b, kv.first.c_str(), v);
    Py_DECREF(v);
  }
  PyObject* t = PyLong_FromLongLong(total);
  PyDict_SetItemString(d, "total", t);
  Py_DECREF(t);
  PyDict_SetItemString(d, "by_verb", a);
  Py_DECREF(a);
  PyDict_SetItemString(d, "by_resource_verb", b);
  Py_DECREF(b);
  PyObject* r = PyLong_FromLongLong(rv);
  PyDict_SetItemString(d, "resourceVersion", r);
  Py_DECREF(r);
  PyObject* q = PyLong_FromLongLong(reqs);
  PyDict_SetItemString(d, "requests", q);
  Py_DECREF(q);
  PyObject* io_d = Py_BuildValue("{s:L,s:L}", "sends", io[0], "turns", io[1]);
  PyDict_SetItemString(d, "io", io_d);  // send() calls and event-loop turns
  Py_DECREF(io_d);
  PyObject* c = Py_BuildValue("{s:d,s:d,s:d,s:d,s:d}", "read_parse", cpu[0] * 1e-9, "verbs", cpu[1] * 1e-9,
                              "fallback", cpu[2] * 1e-9, "frame_write", cpu[3] * 1e-9, "loop", cpu[4] * 1e-9);
  PyDict_SetItemString(d, "server_thread_cpu_s", c);
  Py_DECREF(c);
  PyObject* vc = PyDict_New();
  for (auto& kv : vcpu) {
    PyObject* t = Py_BuildValue("(dL)", kv.second.first * 1e-9, kv.second.second);
    PyDict_SetItemString(vc, kv.first.c_str(), t);
    Py_DECREF(t);
  }
  PyDict_SetItemString(d, "verb_cpu", vc);  // "verb[/sub]:resource" -> (server-thread CPU s, calls)
  PyObject* phd = Py_BuildValue("{s:K,s:K,s:K,s:K,s:K,s:K}", "parse", ph[0], "merge", ph[1], "prepare", ph[2],
                                "finish", ph[3], "emit", ph[4], "reply", ph[5]);
  PyDict_SetItemString(d, "phase_cycles", phd);
  Py_DECREF(phd);
  Py_DECREF(vc);
  PyObject* sa = PyLong_FromLongLong(cpu[5]);
  PyDict_SetItemString(d, "admission_slow_path", sa);
  Py_DECREF(sa);
  return d;
}

// count(group, version, resource, namespace=None) -> int
PyObject* Server_count(Server* self, PyObject* args) {
  const char *g, *v, *r;
  PyObject* ns = Py_None;
  if (!PyArg_ParseTuple(args, "sss|O", &g, &v, &r, &ns)) return nullptr;
  std::string nss;
  const bool has_ns = ns != Py_None;
  if (has_ns) {
    const char* x = PyUnicode_AsUTF8(ns);
    if (!x) return nullptr;
    nss = x;
  }
  Impl* s = self->impl;
  long long n = -1;
  std::string gs(g), vs(v), rs(r);
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    Resource* ri = s->find(gs, vs, rs);
    if (ri) n = static_cast<long long>(s->count(ri, has_ns ? &nss : nullptr));
  }
  Py_END_ALLOW_THREADS
  if (n < 0) {
    PyErr_Format(PyExc_KeyError, "unknown resource %s/%s/%s", g, v, r);
    return nullptr;
  }
  return PyLong_FromLongLong(n);
}

// watchers() -> number of open watches
PyObject* Server_watchers(Server* self, PyObject*) {
  Impl* s = self->impl;
  size_t n = 0;
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    for (auto& kv : s->stores) n += kv.second->watchers.size();
  }
  Py_END_ALLOW_THREADS
  return PyLong_FromSize_t(n);
}

// log_sizes() -> {"group/resource": events held for watch resume}
PyObject* Server_log_sizes(Server* self, PyObject*) {
  Impl* s = self->impl;
  std::vector<std::pair<std::string, size_t>> out;
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> g(s->mu);
    for (auto& kv : s->stores) out.emplace_back(kv.first, kv.second->log.size());
  }
  Py_END_ALLOW_THREADS
  PyObject* d = PyDict_New();
  for (auto& kv : out) {
    PyObject* v = PyLong_FromSize_t(kv.second);
    PyDict_SetItemString(d, kv.first.c_str(), v);
    Py_DECREF(v);
  }
  return d;
}

// unfinished(group, version, resource, namespace) -> [(name, kind, object bytes)]: the objects whose
// status has no completionTime (the bench's training-operator writes go to these)
PyObject* Server_unfinished(Server* self, PyObject* args) {
  const char *g, *v, *r, *ns;
  if (!PyArg_ParseTuple(args, "ssss", &g, &v, &r, &ns)) return nullptr;
  Impl* s = self->impl;
  std::vector<std::tuple<std::string, std::string, std::string>> out;
  bool known = true;
  std::string gs(g), vs(v), rs(r), nss(ns);
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    Resource* ri = s->find(gs, vs, rs);
    if (!ri) {
      known = false;
    } else {
      for (auto& kv : ri->store->data) {
        if (!nss.empty() && kv.first != nss) continue;
        for (auto& ob : kv.second) {
          const Node* st = ob.second->getn("status");
          if (st && st->is_obj()) {
            const Node* ct = st->getn("completionTime");
            if (ct && ct->t == T::Str && !ct->s.empty()) continue;
          }
          std::string enc;
          jdom::write(&enc, ob.second.get());
          out.emplace_back(ob.first, ob.second->str("kind"), std::move(enc));
        }
      }
    }
  }
  Py_END_ALLOW_THREADS
  if (!known) {
    PyErr_Format(PyExc_KeyError, "unknown resource %s/%s/%s", g, v, r);
    return nullptr;
  }
  PyObject* lst = PyList_New(static_cast<Py_ssize_t>(out.size()));
  for (size_t i = 0; i < out.size(); ++i) {
    const auto& t = out[i];
    PyList_SET_ITEM(lst, static_cast<Py_ssize_t>(i),
                    Py_BuildValue("(s#s#y#)", std::get<0>(t).data(), static_cast<Py_ssize_t>(std::get<0>(t).size()),
                                  std::get<1>(t).data(), static_cast<Py_ssize_t>(std::get<1>(t).size()),
                                  std::get<2>(t).data(), static_cast<Py_ssize_t>(std::get<2>(t).size())));
  }
  return lst;
}

// patch_many(group, version, resource, namespace, [(name, merge patch bytes)], subresource="")
//   -> [resourceVersion or None (failed)]: one merge PATCH per item, in one call
PyObject* Server_patch_many(Server* self, PyObject* args) {
  const char *g, *v, *r, *ns, *sub = "";
  PyObject* items;
  if (!PyArg_ParseTuple(args, "ssssO|s", &g, &v, &r, &ns, &items, &sub)) return nullptr;
  PyObject* seq = PySequence_Fast(items, "items: a sequence of (name, body)");
  if (!seq) return nullptr;
  std::vector<std::pair<std::string, std::string>> work;
  const Py_ssize_t n = PySequence_Fast_GET_SIZE(seq);
  work.reserve(static_cast<size_t>(n));
  for (Py_ssize_t i = 0; i < n; ++i) {
    const char *name, *body;
    Py_ssize_t nl, bl;
    if (!PyArg_ParseTuple(PySequence_Fast_GET_ITEM(seq, i), "s#y#", &name, &nl, &body, &bl)) {
      Py_DECREF(seq);
      return nullptr;
    }
    work.emplace_back(std::string(name, static_cast<size_t>(nl)), std::string(body, static_cast<size_t>(bl)));
  }
  Py_DECREF(seq);
  Impl* s = self->impl;
  std::vector<std::string> rvs(work.size());
  std::vector<bool> ok(work.size(), false);
  bool known = true;
  std::string gs(g), vs(v), rs(r), nss(ns), subs(sub);
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    Resource* ri = s->find(gs, vs, rs);
    if (!ri) {
      known = false;
    } else {
      for (size_t i = 0; i < work.size(); ++i) {
        Ref body = jdom::parse(work[i].second.data(), work[i].second.size());
        if (!body) continue;
        ApiErr err;
        Ref out = s->v_patch(ri, nss, work[i].first, body, "merge", subs, &err);
        if (out) {
          rvs[i] = meta_str(out.get(), "resourceVersion");
          ok[i] = true;
        }
      }
    }
    if (!s->running || std::this_thread::get_id() != s->thread.get_id()) s->end_of_turn();
  }
  Py_END_ALLOW_THREADS
  if (!known) {
    PyErr_Format(PyExc_KeyError, "unknown resource %s/%s/%s", g, v, r);
    return nullptr;
  }
  PyObject* lst = PyList_New(static_cast<Py_ssize_t>(work.size()));
  for (size_t i = 0; i < work.size(); ++i) {
    PyObject* x = ok[i] ? PyUnicode_FromStringAndSize(rvs[i].data(), static_cast<Py_ssize_t>(rvs[i].size()))
                        : (Py_INCREF(Py_None), Py_None);
    PyList_SET_ITEM(lst, static_cast<Py_ssize_t>(i), x);
  }
  return lst;
}

// patch_unfinished(group, version, resource, namespace, template, placeholder, subresource="",
//   per_turn=0) -> int: one merge PATCH per object whose status has no completionTime, its body
//   the template with `placeholder` replaced by the object's name -- the bench's "every job
//   finishes" write, without a Python round trip per job.  per_turn > 0 on a running server:
//   the patches are queued and the server thread applies that many per loop turn, between the
//   turns serving other clients (returns the number queued)
// `t` with every `ph` inside its strings replaced by `name` (keys untouched): a node whose
// subtree holds no placeholder is shared, not copied
Ref subst(const Ref& t, const std::string& ph, const std::string& name) {
  switch (t->t) {
    case T::Str: {
      if (t->s.find(ph.data(), 0, ph.size()) == jdom::jstr::npos) return t;
      std::string v;
      size_t pos = 0;
      const std::string_view sv(t->s);
      while (true) {
        const size_t hit = sv.find(ph, pos);
        if (hit == std::string_view::npos) {
          v.append(sv.substr(pos));
          break;
        }
        v.append(sv.substr(pos, hit - pos));
        v.append(name);
        pos = hit + ph.size();
      }
      return jdom::mk_str(v);
    }
    case T::Arr: {
      Ref out;
      for (size_t i = 0; i < t->a.size(); ++i) {
        Ref c = subst(t->a[i], ph, name);
        if (c == t->a[i]) continue;
        if (!out) out = jdom::shallow(t.get());
        out->a[i] = std::move(c);
      }
      return out ? out : t;
    }
    case T::Obj: {
      Ref out;
      for (size_t i = 0; i < t->o.size(); ++i) {
        Ref c = subst(t->o[i].second, ph, name);
        if (c == t->o[i].second) continue;
        if (!out) out = jdom::shallow(t.get());
        out->o[i].second = std::move(c);
      }
      return out ? out : t;
    }
    default: return t;
  }
}

PyObject* Server_patch_unfinished(Server* self, PyObject* args) {
  const char *g, *v, *r, *ns, *tmpl, *ph, *sub = "";
  Py_ssize_t tl, pl, per_turn = 0;
  if (!PyArg_ParseTuple(args, "sssss#s#|sn", &g, &v, &r, &ns, &tmpl, &tl, &ph, &pl, &sub, &per_turn)) return nullptr;
  Impl* s = self->impl;
  long long n = 0;
  bool known = true;
  std::string gs(g), vs(v), rs(r), nss(ns), subs(sub), ts(tmpl, static_cast<size_t>(tl)),
      phs(ph, static_cast<size_t>(pl));
  Py_BEGIN_ALLOW_THREADS
  {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    Resource* ri = s->find(gs, vs, rs);
    if (!ri || phs.empty()) {
      known = false;
    } else {
      // the targets first: the patches change the store being walked
      std::vector<std::pair<std::string, std::string>> todo;
      for (auto& kv : ri->store->data) {
        if (!nss.empty() && kv.first != nss) continue;
        for (auto& ob : kv.second) {
          const Node* st = ob.second->getn("status");
          if (st && st->is_obj()) {
            const Node* ct = st->getn("completionTime");
            if (ct && ct->t == T::Str && !ct->s.empty()) continue;
          }
          todo.emplace_back(kv.first, ob.first);
        }
      }
      // the template parsed once; each job's patch copies only the nodes whose strings hold
      // the placeholder (a condition's message), the rest is shared
      Ref tree = jdom::parse(ts.data(), ts.size());
      if (tree && per_turn > 0 && s->running) {
        // queued: the server thread applies `per_turn` of them per loop turn (run_pending_patches)
        n = static_cast<long long>(todo.size());
        Impl::PendingPatches p;
        p.g = gs;
        p.v = vs;
        p.r = rs;
        p.sub = subs;
        p.ph = phs;
        p.tree = tree;
        p.todo = std::move(todo);
        p.per_turn = static_cast<size_t>(per_turn);
        if (n) s->pending_patches.push_back(std::move(p));
        if (std::this_thread::get_id() != s->thread.get_id()) s->wake();
      } else {
        for (const auto& t : todo) {
          if (!tree) break;
          Ref patch = subst(tree, phs, t.second);
          ApiErr err;
          if (s->v_patch(ri, t.first, t.second, patch, "merge", subs, &err)) ++n;
        }
      }
    }
    if (!s->running || std::this_thread::get_id() != s->thread.get_id()) s->end_of_turn();
  }
  Py_END_ALLOW_THREADS
  if (!known) {
    PyErr_Format(PyExc_KeyError, "unknown resource %s/%s/%s (or an empty placeholder)", g, v, r);
    return nullptr;
  }
  return PyLong_FromLongLong(n);
}

// ---------------------------------------------------------------------- sampling profiler
// There is no perf on the benchmark boxes: a SIGPROF timer on process CPU time samples the stack
// of whichever thread runs (the server thread, in a benchmark), and profile_stop() returns the
// stacks as (module path, offset) frames -- tests/scripts resolve them with addr2line.
namespace prof {
constexpr size_t kCap = 1 << 21;  // frames
std::atomic<bool> on{false};
uint64_t* frames = nullptr;       // stacks, each ended by a 0
std::atomic<size_t> used{0};
std::atomic<size_t> dropped{0};
timer_t timer;
bool has_timer = false;

void handler(int, siginfo_t*, void*) {
  if (!on.load(std::memory_order_relaxed)) return;
  void* buf[48];
  const int n = backtrace(buf, 48);
  const size_t need = static_cast<size_t>(n) + 1;
  const size_t at = used.fetch_add(need, std::memory_order_relaxed);
  if (at + need > kCap) {
    dropped.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  // [0] is this handler and [1] the kernel's signal trampoline: the interrupted frame is [2]
  size_t k = at;
  for (int i = 2; i < n; ++i) frames[k++] = reinterpret_cast<uint64_t>(buf[i]);
  while (k < at + need) frames[k++] = 0;
}
}  // namespace prof

// profile_start(interval_s=0.0005)
// With the server thread running, a CLOCK_MONOTONIC timer signals that thread alone (hrtimer
// resolution: process-CPU itimers tick at the kernel's HZ, 100-250 samples a second); samples
// that land in epoll_wait are the thread idling, which the report counts apart.
PyObject* Server_profile_start(Server* self, PyObject* args) {
  double interval = 0.0005;
  if (!PyArg_ParseTuple(args, "|d", &interval)) return nullptr;
  if (!(interval > 0.0) || interval > 1.0) {
    PyErr_SetString(PyExc_ValueError, "interval_s must be in (0, 1]");
    return nullptr;
  }
  if (!prof::frames) prof::frames = new uint64_t[prof::kCap];
  void* warm[4];
  backtrace(warm, 4);  // the unwinder loads (and allocates) on its first use: not in the handler
  prof::used.store(0);
  prof::dropped.store(0);
  struct sigaction sa;
  std::memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = prof::handler;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  sigaction(SIGPROF, &sa, nullptr);
  prof::on.store(true);
  if (prof::has_timer) {  // started again without a stop: the old timer goes first
    timer_delete(prof::timer);
    prof::has_timer = false;
  }
  const pid_t tid = self->impl->running ? self->impl->loop_tid.load() : 0;
  if (tid > 0) {
    struct sigevent sev;
    std::memset(&sev, 0, sizeof sev);
    sev.sigev_notify = SIGEV_THREAD_ID;
    sev.sigev_signo = SIGPROF;
    sev._sigev_un._tid = tid;
    if (timer_create(CLOCK_MONOTONIC, &sev, &prof::timer) == 0) {
      prof::has_timer = true;
      struct itimerspec its;
      its.it_interval.tv_sec = static_cast<time_t>(interval);
      its.it_interval.tv_nsec = static_cast<long>((interval - static_cast<double>(its.it_interval.tv_sec)) * 1e9);
      its.it_value = its.it_interval;
      timer_settime(prof::timer, 0, &its, nullptr);
      Py_RETURN_NONE;
    }
  }
  struct itimerval it;
  it.it_interval.tv_sec = static_cast<time_t>(interval);
  it.it_interval.tv_usec = static_cast<suseconds_t>((interval - static_cast<double>(it.it_interval.tv_sec)) * 1e6);
  it.it_value = it.it_interval;
  setitimer(ITIMER_PROF, &it, nullptr);
  Py_RETURN_NONE;
}

// profile_stop() -> (stacks: [[(module, offset), ...] innermost first], dropped)
PyObject* Server_profile_stop(Server*, PyObject*) {
  if (prof::has_timer) {
    timer_delete(prof::timer);
    prof::has_timer = false;
  }
  struct itimerval it;
  std::memset(&it, 0, sizeof it);
  setitimer(ITIMER_PROF, &it, nullptr);
  prof::on.store(false);
  const size_t n = std::min(prof::used.load(), prof::kCap);
  PyObject* stacks = PyList_New(0);
  PyObject* cur = PyList_New(0);
  std::unordered_map<uint64_t, std::pair<std::string, uint64_t>> memo;
  for (size_t i = 0; i < n && prof::frames; ++i) {
    const uint64_t a = prof::frames[i];
    if (a == 0) {
      if (PyList_GET_SIZE(cur) > 0) PyList_Append(stacks, cur);
      Py_DECREF(cur);
      cur = PyList_New(0);
      continue;
    }
    auto it2 = memo.find(a);
    if (it2 == memo.end()) {
      Dl_info info;
      std::pair<std::string, uint64_t> v("?", a);
      if (dladdr(reinterpret_cast<void*>(a), &info) && info.dli_fname) {
        v.first = info.dli_fname;
        v.second = a - reinterpret_cast<uint64_t>(info.dli_fbase) - 1;  // the call, not the return
      }
      it2 = memo.emplace(a, v).first;
    }
    PyObject* t = Py_BuildValue("(sK)", it2->second.first.c_str(),
                                static_cast<unsigned long long>(it2->second.second));
    PyList_Append(cur, t);
    Py_DECREF(t);
  }
  Py_DECREF(cur);
  return Py_BuildValue("(Nn)", stacks, static_cast<Py_ssize_t>(prof::dropped.load()));
}

PyObject* Server_port(Server* self, void*) { return PyLong_FromLong(self->impl->port); }

PyMethodDef Server_methods[] = {
    {"request", reinterpret_cast<PyCFunction>(Server_request), METH_VARARGS | METH_KEYWORDS,
     "request(method, path, query='', body=b'', content_type='', accept='') -> (status, body): one REST call "
     "served in-process (what an HTTP request to the same path would get)"},
    {"start", reinterpret_cast<PyCFunction>(Server_start), METH_VARARGS | METH_KEYWORDS,
     "start(host='127.0.0.1', port=0, certfile='', keyfile='') -> port: serve on the server thread"},
    {"stop", reinterpret_cast<PyCFunction>(Server_stop), METH_NOARGS, "end every watch and stop serving"},
    {"set_clock", reinterpret_cast<PyCFunction>(Server_set_clock), METH_O, "set the server clock (ns since epoch)"},
    {"now_ns", reinterpret_cast<PyCFunction>(Server_now_ns), METH_NOARGS, "the server clock"},
    {"set_latency", reinterpret_cast<PyCFunction>(Server_set_latency), METH_O,
     "per-verb injected latency in seconds ('*' default, 'list_per_object')"},
    {"clear_latency", reinterpret_cast<PyCFunction>(Server_clear_latency), METH_NOARGS, "no injected latency"},
    {"set_fallback", reinterpret_cast<PyCFunction>(Server_set_fallback), METH_O,
     "fallback(method, path, query, headers, body) -> (status, body[, content_type[, headers]]) | None"},
    {"stats", reinterpret_cast<PyCFunction>(Server_stats), METH_NOARGS, "request accounting"},
    {"count", reinterpret_cast<PyCFunction>(Server_count), METH_VARARGS, "objects of a resource"},
    {"watchers", reinterpret_cast<PyCFunction>(Server_watchers), METH_NOARGS, "open watches"},
    {"profile_start", reinterpret_cast<PyCFunction>(Server_profile_start), METH_VARARGS,
     "profile_start(interval_s=0.0005): sample stacks on process CPU time (SIGPROF)"},
    {"profile_stop", reinterpret_cast<PyCFunction>(Server_profile_stop), METH_NOARGS,
     "profile_stop() -> (stacks of (module, offset) frames, innermost first; dropped samples)"},
    {"log_sizes", reinterpret_cast<PyCFunction>(Server_log_sizes), METH_NOARGS,
     "events kept per resource for watch resume"},
    {"unfinished", reinterpret_cast<PyCFunction>(Server_unfinished), METH_VARARGS,
     "unfinished(group, version, resource, namespace) -> [(name, kind, bytes)] without status.completionTime"},
    {"patch_unfinished", reinterpret_cast<PyCFunction>(Server_patch_unfinished), METH_VARARGS,
     "patch_unfinished(group, version, resource, namespace, template, placeholder, subresource='', per_turn=0) -> int "
     "(per_turn > 0 on a running server: queued, that many applied per loop turn)"},
    {"patch_many", reinterpret_cast<PyCFunction>(Server_patch_many), METH_VARARGS,
     "patch_many(group, version, resource, namespace, [(name, body)], subresource='') -> [resourceVersion|None]"},
    {nullptr, nullptr, 0, nullptr}};

PyGetSetDef Server_getset[] = {{"port", reinterpret_cast<getter>(Server_port), nullptr, "bound port", nullptr},
                               {nullptr, nullptr, nullptr, nullptr, nullptr}};

PyTypeObject ServerType = {PyVarObject_HEAD_INIT(nullptr, 0)};

PyModuleDef moddef = {PyModuleDef_HEAD_INIT, "_apiserverd",
                      "The fake Kubernetes apiserver's store, admission, watch fan-out and HTTP front end, native "
                      "(ops/csrc/apiserverd.cpp).",
                      -1, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__apiserverd(void) {
  ServerType.tp_name = "_apiserverd.Server";
  ServerType.tp_basicsize = sizeof(Server);
  ServerType.tp_flags = Py_TPFLAGS_DEFAULT;
  ServerType.tp_new = Server_new;
  ServerType.tp_init = reinterpret_cast<initproc>(Server_init);
  ServerType.tp_dealloc = reinterpret_cast<destructor>(Server_dealloc);
  ServerType.tp_methods = Server_methods;
  ServerType.tp_getset = Server_getset;
  ServerType.tp_doc = "Server(now_ns=0, watch_window=200000, bookmark_interval=60.0)";
  if (PyType_Ready(&ServerType) < 0) return nullptr;
  PyObject* m = PyModule_Create(&moddef);
  if (!m) return nullptr;
  Py_INCREF(&ServerType);
  PyModule_AddObject(m, "Server", reinterpret_cast<PyObject*>(&ServerType));
  return m;
}
#endif  // APISERVERD_STANDALONE
