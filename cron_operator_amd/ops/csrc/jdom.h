// Immutable, reference-counted JSON trees for the native fake apiserver (`_apiserverd`).
//
// The Python fake apiserver (apiserver/server.py) stores objects as dicts it never mutates in
// place, so a status write shares the stored object's spec and a tombstone shares everything but
// its metadata.  This is the same model in C++: a stored JNode is never changed again, writes
// build new nodes that point at the untouched subtrees of the old ones (RFC 7386 merge patch
// keeps the path of every shared subtree), and each container node caches its serialised bytes
// once written -- so a status PATCH re-encodes the changed members and splices in the cached
// bytes of the rest, like `_fastjson.dumpb_shared` does for the Python store.
//
// Reference counts are not atomic: every tree is touched by the server thread only (Python
// entry points take the server's lock first).
//
// Memory: a write builds tens of nodes, member vectors, strings and 1-4 KiB encodings, and
// retiring a version frees as many.  glibc's malloc cost as much as the JSON work itself (gprof
// of the standalone driver: _int_malloc + malloc_consolidate + _int_free ~40%), so nodes come
// from a free list and every container and string of a tree from size-class free lists
// (PoolAlloc: thread-local LIFO lists, no header -- the containers pass the size back).  Only
// this header's types use them: nothing crosses into libstdc++'s own allocations.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace jdom {

namespace pool {

constexpr size_t kMax = 16384;  // larger blocks go to operator new
constexpr int kClasses = 48;
constexpr uint32_t kMaxFree = 1u << 15;  // spare blocks kept per class and thread ...
constexpr size_t kMaxFreeBytes = 4u << 20;  // ... and at most this many bytes of them

struct Tables {
  size_t size[kClasses] = {};
  uint32_t cap[kClasses] = {};
  unsigned char by16[(kMax >> 4) + 1] = {};
  int n = 0;
  Tables() {
    size_t s = 16;
    while (s < kMax && n < kClasses - 1) {
      size[n++] = s;
      s = s < 256 ? s + 16 : (s + s / 4 + 15) / 16 * 16;
    }
    size[n++] = kMax;
    // JDOM_POOL=0: no spare blocks at all (every block back to malloc: the soak's A/B arm)
    const char* env = std::getenv("JDOM_POOL");
    const bool off = env && env[0] == '0';
    for (int i = 0; i < n; ++i)
      cap[i] = off ? 0u : static_cast<uint32_t>(std::max<size_t>(64, std::min<size_t>(kMaxFree, kMaxFreeBytes / size[i])));
    int c = 0;
    for (size_t i = 0; i <= (kMax >> 4); ++i) {
      while (size[c] < (i << 4)) ++c;
      by16[i] = static_cast<unsigned char>(c);
    }
  }
};

inline const Tables& tables() {
  static const Tables t;
  return t;
}

struct Lists {
  void* head[kClasses] = {};
  uint32_t count[kClasses] = {};
};

inline Lists& lists() {
  static thread_local Lists l;
  return l;
}

inline void* alloc(size_t n) {
  if (n > kMax) return ::operator new(n);
  const Tables& t = tables();
  const unsigned c = t.by16[(n + 15) >> 4];
  Lists& l = lists();
  if (void* b = l.head[c]) {
    l.head[c] = *static_cast<void**>(b);
    --l.count[c];
    return b;
  }
  return ::operator new(t.size[c]);
}

inline void release(void* p, size_t n) noexcept {
  if (!p) return;
  if (n > kMax) {
    ::operator delete(p);
    return;
  }
  const Tables& t = tables();
  const unsigned c = t.by16[(n + 15) >> 4];
  Lists& l = lists();
  if (l.count[c] >= t.cap[c]) {
    ::operator delete(p);
    return;
  }
  *static_cast<void**>(p) = l.head[c];
  l.head[c] = p;
  ++l.count[c];
}

}  // namespace pool

template <class T>
struct PoolAlloc {
  using value_type = T;
  PoolAlloc() noexcept = default;
  template <class U>
  PoolAlloc(const PoolAlloc<U>&) noexcept {}  // NOLINT: rebinding
  T* allocate(size_t n) { return static_cast<T*>(pool::alloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) noexcept { pool::release(p, n * sizeof(T)); }
  template <class U>
  bool operator==(const PoolAlloc<U>&) const noexcept { return true; }
  template <class U>
  bool operator!=(const PoolAlloc<U>&) const noexcept { return false; }
};

using jstr = std::basic_string<char, std::char_traits<char>, PoolAlloc<char>>;

enum class T : uint8_t { Null, False, True, Num, Str, Arr, Obj };

struct Node;

// intrusive pointer (single-threaded refcount)
class Ref {
 public:
  Ref() = default;
  Ref(Node* n);  // NOLINT: implicit from a fresh node
  Ref(const Ref& o);
  Ref(Ref&& o) noexcept : p_(o.p_) { o.p_ = nullptr; }
  ~Ref();
  Ref& operator=(const Ref& o);
  Ref& operator=(Ref&& o) noexcept;
  Node* operator->() const { return p_; }
  Node& operator*() const { return *p_; }
  Node* get() const { return p_; }
  explicit operator bool() const { return p_ != nullptr; }
  bool operator==(const Ref& o) const { return p_ == o.p_; }
  bool operator!=(const Ref& o) const { return p_ != o.p_; }

 private:
  Node* p_ = nullptr;
};

using Member = std::pair<jstr, Ref>;
using RefVec = std::vector<Ref, PoolAlloc<Ref>>;
using MemberVec = std::vector<Member, PoolAlloc<Member>>;

// Nodes come and go by the tens per request (a parsed body, merge results, tombstones): a free
// list keeps them out of malloc, where they cost more than the JSON work itself (gprof of the
// standalone driver: _int_malloc + malloc_consolidate + _int_free were ~45% of the server's CPU).
// Not thread-safe: every tree is built and dropped under the server's lock.
struct NodePool {
  struct Free {
    Free* next;
  };
  Free* head = nullptr;
  size_t cached = 0;
  size_t cap = 1u << 18;  // at most 256K spare nodes (~32 MiB); JDOM_POOL=0: none
  NodePool() {
    const char* env = std::getenv("JDOM_POOL");
    if (env && env[0] == '0') cap = 0;
  }
  static NodePool& get() {
    static NodePool p;
    return p;
  }
};

struct Node {
  static void* operator new(size_t n) {
    NodePool& p = NodePool::get();
    if (p.head) {
      NodePool::Free* f = p.head;
      p.head = f->next;
      --p.cached;
      return f;
    }
    return ::operator new(n);
  }
  static void operator delete(void* ptr) {
    NodePool& p = NodePool::get();
    if (p.cached >= p.cap) {
      ::operator delete(ptr);
      return;
    }
    NodePool::Free* f = static_cast<NodePool::Free*>(ptr);
    f->next = p.head;
    p.head = f;
    ++p.cached;
  }

  uint32_t rc = 0;
  uint32_t hint = 0;  // a container's expected encoded size (its previous version's), for reserve
  T t = T::Null;
  // passed schema admission at its path (apiserver admission skips such subtrees)
  bool admitted = false;
  jstr s;                     // Str: the value (unescaped); Num: the lexeme as sent
  RefVec a;                   // Arr
  MemberVec o;                // Obj, insertion order
  jstr enc;                   // Arr/Obj: cached serialisation ("" = not cached)

  explicit Node(T t_) : t(t_) {}

  bool is_obj() const { return t == T::Obj; }
  bool is_arr() const { return t == T::Arr; }
  bool is_str() const { return t == T::Str; }

  // object member lookup (objects are small: a linear scan beats hashing)
  const Ref* get(const char* k, size_t n) const {
    for (const auto& m : o)
      if (m.first.size() == n && std::memcmp(m.first.data(), k, n) == 0) return &m.second;
    return nullptr;
  }
  const Ref* get(std::string_view k) const { return get(k.data(), k.size()); }
  const Ref* get(const char* k) const { return get(k, std::strlen(k)); }
  Node* getn(const char* k) const {
    const Ref* r = get(k);
    return r ? r->get() : nullptr;
  }
  // string member value ("" when absent or not a string)
  std::string_view str(const char* k) const;
  // set/replace a member (the node must be private to the caller: fresh, not stored)
  void set(std::string_view k, Ref v) {
    enc.clear();
    for (auto& m : o)
      if (std::string_view(m.first) == k) {
        m.second = std::move(v);
        return;
      }
    o.emplace_back(jstr(k), std::move(v));
  }
  bool erase(const char* k) {
    const size_t n = std::strlen(k);
    for (size_t i = 0; i < o.size(); ++i)
      if (o[i].first.size() == n && std::memcmp(o[i].first.data(), k, n) == 0) {
        o.erase(o.begin() + static_cast<long>(i));
        enc.clear();
        return true;
      }
    return false;
  }
};

inline Ref::Ref(Node* n) : p_(n) {
  if (p_) ++p_->rc;
}
inline Ref::Ref(const Ref& o) : p_(o.p_) {
  if (p_) ++p_->rc;
}
inline Ref::~Ref() {
  if (p_ && --p_->rc == 0) delete p_;
}
inline Ref& Ref::operator=(const Ref& o) {
  if (o.p_) ++o.p_->rc;
  if (p_ && --p_->rc == 0) delete p_;
  p_ = o.p_;
  return *this;
}
inline Ref& Ref::operator=(Ref&& o) noexcept {
  if (this != &o) {
    if (p_ && --p_->rc == 0) delete p_;
    p_ = o.p_;
    o.p_ = nullptr;
  }
  return *this;
}

inline std::string_view Node::str(const char* k) const {
  const Ref* r = get(k);
  return (r && (*r)->t == T::Str) ? std::string_view((*r)->s) : std::string_view();
}

inline Ref mk_str(std::string_view v) {
  Node* n = new Node(T::Str);
  n->s.assign(v.data(), v.size());
  return Ref(n);
}
inline Ref mk_num(long long v) {
  Node* n = new Node(T::Num);
  char buf[24];
  const int len = snprintf(buf, sizeof buf, "%lld", v);
  n->s.assign(buf, static_cast<size_t>(len));
  return Ref(n);
}
inline Ref mk_obj() { return Ref(new Node(T::Obj)); }
inline Ref mk_arr() { return Ref(new Node(T::Arr)); }
inline Ref mk_null() { return Ref(new Node(T::Null)); }
inline Ref mk_bool(bool b) { return Ref(new Node(b ? T::True : T::False)); }

// shallow copy: a private node sharing the children (copy-on-write of one level)
inline Ref shallow(const Node* n) {
  Node* c = new Node(n->t);
  c->hint = static_cast<uint32_t>(n->enc.empty() ? n->hint : n->enc.size());
  c->s = n->s;
  c->a = n->a;
  c->o = n->o;
  return Ref(c);
}

// ------------------------------------------------------------------ parse

// The parser keeps the source bytes of containers at depth 1 and 2 (at least kSpanMin long) as
// their encoding: the body a client sent is valid JSON for the node it decoded to, so a subtree
// that reaches the store unchanged -- a job's spec, a status patch's conditions or history -- is
// never encoded again.  Whoever mutates such a node clears its enc *and its ancestors'*
// (Node::set/erase clear the node's own; apiserverd's admission reports changes upward).
constexpr size_t kSpanMin = 24;

class Parser {
 public:
  Parser(const char* b, size_t n) : p_(b), e_(b + n) {}
  // nullptr Ref + err() on malformed input
  Ref parse() {
    ws();
    Ref r = value(0);
    astack_.clear();  // a failed parse leaves partial containers on the shared stacks
    ostack_.clear();
    if (!r) return r;
    ws();
    if (p_ != e_) return fail("extra data after JSON value");
    return r;
  }
  const std::string& err() const { return err_; }

 private:
  const char* p_;
  const char* e_;
  std::string err_;

  Ref fail(const char* m) {
    if (err_.empty()) err_ = m;
    return Ref();
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  Ref value(int depth) {
    if (depth > 512) return fail("nesting too deep");
    if (p_ >= e_) return fail("unexpected end of JSON");
    switch (*p_) {
      case '{': return object(depth);
      case '[': return array(depth);
      case '"': {
        Node* n = new Node(T::Str);
        Ref r(n);
        if (!string(&n->s)) return Ref();
        return r;
      }
      case 't':
        if (e_ - p_ >= 4 && std::memcmp(p_, "true", 4) == 0) {
          p_ += 4;
          return mk_bool(true);
        }
        return fail("invalid literal");
      case 'f':
        if (e_ - p_ >= 5 && std::memcmp(p_, "false", 5) == 0) {
          p_ += 5;
          return mk_bool(false);
        }
        return fail("invalid literal");
      case 'n':
        if (e_ - p_ >= 4 && std::memcmp(p_, "null", 4) == 0) {
          p_ += 4;
          return mk_null();
        }
        return fail("invalid literal");
      default: return number();
    }
  }
  Ref number() {
    const char* b = p_;
    if (p_ < e_ && *p_ == '-') ++p_;
    if (p_ >= e_ || *p_ < '0' || *p_ > '9') return fail("invalid value");
    if (*p_ == '0') {
      ++p_;
    } else {
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    if (p_ < e_ && *p_ == '.') {
      ++p_;
      if (p_ >= e_ || *p_ < '0' || *p_ > '9') return fail("invalid number");
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
      ++p_;
      if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
      if (p_ >= e_ || *p_ < '0' || *p_ > '9') return fail("invalid number");
      while (p_ < e_ && *p_ >= '0' && *p_ <= '9') ++p_;
    }
    Node* n = new Node(T::Num);
    n->s.assign(b, static_cast<size_t>(p_ - b));
    return Ref(n);
  }
  static void put_utf8(jstr* out, unsigned cp) {
    if (cp < 0x80) {
      out->push_back(static_cast<char>(cp));
    } else if (cp < 0x800) {
      out->push_back(static_cast<char>(0xC0 | (cp >> 6)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      out->push_back(static_cast<char>(0xE0 | (cp >> 12)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    } else {
      out->push_back(static_cast<char>(0xF0 | (cp >> 18)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
      out->push_back(static_cast<char>(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(unsigned* out) {
    if (e_ - p_ < 4) return false;
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = p_[i];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= static_cast<unsigned>(c - '0');
      else if (c >= 'a' && c <= 'f') v |= static_cast<unsigned>(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= static_cast<unsigned>(c - 'A' + 10);
      else return false;
    }
    p_ += 4;
    *out = v;
    return true;
  }
  // bytes that end a plain run inside a string: the quote, a backslash, control characters
  static const bool* special() {
    static const struct T {
      bool t[256];
      T() : t() {
        for (int i = 0; i < 0x20; ++i) t[i] = true;
        t[static_cast<unsigned char>('"')] = true;
        t[static_cast<unsigned char>('\\')] = true;
      }
    } tab;
    return tab.t;
  }

  bool string(jstr* out) {
    ++p_;  // opening quote
    const bool* sp = special();
    const char* run = p_;
    while (p_ < e_ && !sp[static_cast<unsigned char>(*p_)]) ++p_;
    if (p_ < e_ && *p_ == '"') {  // no escapes: one copy at its final size
      out->assign(run, static_cast<size_t>(p_ - run));
      ++p_;
      return true;
    }
    out->assign(run, static_cast<size_t>(p_ - run));
    run = p_;
    while (true) {
      if (p_ >= e_) {
        fail("unterminated string");
        return false;
      }
      const unsigned char c = static_cast<unsigned char>(*p_);
      if (c == '"') {
        out->append(run, static_cast<size_t>(p_ - run));
        ++p_;
        return true;
      }
      if (c < 0x20) {
        fail("invalid control character in string");
        return false;
      }
      if (c != '\\') {
        ++p_;
        continue;
      }
      out->append(run, static_cast<size_t>(p_ - run));
      ++p_;
      if (p_ >= e_) {
        fail("unterminated string");
        return false;
      }
      const char esc = *p_++;
      switch (esc) {
        case '"': out->push_back('"'); break;
        case '\\': out->push_back('\\'); break;
        case '/': out->push_back('/'); break;
        case 'b': out->push_back('\b'); break;
        case 'f': out->push_back('\f'); break;
        case 'n': out->push_back('\n'); break;
        case 'r': out->push_back('\r'); break;
        case 't': out->push_back('\t'); break;
        case 'u': {
          unsigned cp;
          if (!hex4(&cp)) {
            fail("invalid \\u escape");
            return false;
          }
          if (cp >= 0xD800 && cp < 0xDC00 && e_ - p_ >= 6 && p_[0] == '\\' && p_[1] == 'u') {
            const char* save = p_;
            p_ += 2;
            unsigned lo;
            if (hex4(&lo) && lo >= 0xDC00 && lo < 0xE000) {
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            } else {
              p_ = save;
            }
          }
          put_utf8(out, cp);
          break;
        }
        default: fail("invalid escape"); return false;
      }
      run = p_;
    }
  }
  // containers collect their children on a scratch stack, then take them at exact capacity; the
  // stacks live as long as the thread (a parse would otherwise regrow them from empty)
  static std::vector<Ref>& astack() {
    static thread_local std::vector<Ref> v;
    return v;
  }
  static std::vector<Member>& ostack() {
    static thread_local std::vector<Member> v;
    return v;
  }
  std::vector<Ref>& astack_ = astack();
  std::vector<Member>& ostack_ = ostack();
  size_t dups_ = 0;  // repeated keys seen so far: a span holding one is not its node's encoding

  Ref array(int depth) {
    const char* start = p_;
    const size_t dups0 = dups_;
    ++p_;
    Node* n = new Node(T::Arr);
    Ref r(n);
    ws();
    if (p_ < e_ && *p_ == ']') {
      ++p_;
      return r;
    }
    const size_t base = astack_.size();
    while (true) {
      ws();
      Ref v = value(depth + 1);
      if (!v) return Ref();
      astack_.push_back(std::move(v));
      ws();
      if (p_ >= e_) return fail("unterminated array");
      if (*p_ == ',') {
        ++p_;
        continue;
      }
      if (*p_ == ']') {
        ++p_;
        n->a.reserve(astack_.size() - base);
        for (size_t i = base; i < astack_.size(); ++i) n->a.push_back(std::move(astack_[i]));
        astack_.resize(base);
        if ((depth == 1 || depth == 2) && static_cast<size_t>(p_ - start) >= kSpanMin && dups_ == dups0)
          n->enc.assign(start, p_);
        return r;
      }
      return fail("expected ',' or ']'");
    }
  }
  Ref object(int depth) {
    const char* start = p_;
    const size_t dups0 = dups_;
    ++p_;
    Node* n = new Node(T::Obj);
    Ref r(n);
    ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
      return r;
    }
    const size_t base = ostack_.size();
    while (true) {
      ws();
      if (p_ >= e_ || *p_ != '"') return fail("expected property name");
      ostack_.emplace_back();
      if (!string(&ostack_.back().first)) return Ref();
      ws();
      if (p_ >= e_ || *p_ != ':') return fail("expected ':'");
      ++p_;
      ws();
      Ref v = value(depth + 1);
      if (!v) return Ref();
      // a repeated key keeps the last value, as Python's json does
      const jstr& k = ostack_.back().first;
      bool dup = false;
      for (size_t i = base; i + 1 < ostack_.size(); ++i)
        if (ostack_[i].first == k) {
          ostack_[i].second = std::move(v);
          dup = true;
          break;
        }
      if (dup) {
        ostack_.pop_back();
        ++dups_;
      } else {
        ostack_.back().second = std::move(v);
      }
      ws();
      if (p_ >= e_) return fail("unterminated object");
      if (*p_ == ',') {
        ++p_;
        continue;
      }
      if (*p_ == '}') {
        ++p_;
        n->o.reserve(ostack_.size() - base);
        for (size_t i = base; i < ostack_.size(); ++i) n->o.push_back(std::move(ostack_[i]));
        ostack_.resize(base);
        if ((depth == 1 || depth == 2) && static_cast<size_t>(p_ - start) >= kSpanMin && dups_ == dups0)
          n->enc.assign(start, p_);
        return r;
      }
      return fail("expected ',' or '}'");
    }
  }
};

inline Ref parse(const char* b, size_t n, std::string* err = nullptr) {
  Parser p(b, n);
  Ref r = p.parse();
  if (!r && err) *err = p.err();
  return r;
}

// ------------------------------------------------------------------ serialise

template <class S>
inline void put_string(S* out, std::string_view s) {
  static const char* hex = "0123456789abcdef";
  out->push_back('"');
  const char* b = s.data();
  const char* e = b + s.size();
  const char* run = b;
  for (const char* p = b; p < e; ++p) {
    const unsigned char c = static_cast<unsigned char>(*p);
    if (c >= 0x20 && c != '"' && c != '\\') continue;
    out->append(run, static_cast<size_t>(p - run));
    switch (c) {
      case '"': out->append("\\\""); break;
      case '\\': out->append("\\\\"); break;
      case '\n': out->append("\\n"); break;
      case '\r': out->append("\\r"); break;
      case '\t': out->append("\\t"); break;
      case '\b': out->append("\\b"); break;
      case '\f': out->append("\\f"); break;
      default:
        out->append("\\u00");
        out->push_back(hex[c >> 4]);
        out->push_back(hex[c & 15]);
    }
    run = p + 1;
  }
  out->append(run, static_cast<size_t>(e - run));
  out->push_back('"');
}

// Write `n`.  Containers at depth < cache_depth keep their bytes (n->enc) for the next write --
// the object itself and its top-level members, so a status write re-encodes status and metadata
// and splices in the cached spec; a container that already has them is appended as is.
template <class S>
inline void write(S* out, Node* n, int depth = 0, int cache_depth = 2);

template <class S>
inline void write_body(S* out, Node* n, int depth, int cache_depth) {
  if (n->t == T::Arr) {
    out->push_back('[');
    bool first = true;
    for (const Ref& v : n->a) {
      if (!first) out->push_back(',');
      first = false;
      write(out, v.get(), depth + 1, cache_depth);
    }
    out->push_back(']');
  } else {
    out->push_back('{');
    bool first = true;
    for (const Member& m : n->o) {
      if (!first) out->push_back(',');
      first = false;
      put_string(out, m.first);
      out->push_back(':');
      write(out, m.second.get(), depth + 1, cache_depth);
    }
    out->push_back('}');
  }
}

template <class S>
inline void write(S* out, Node* n, int depth, int cache_depth) {
  switch (n->t) {
    case T::Null: out->append("null"); return;
    case T::True: out->append("true"); return;
    case T::False: out->append("false"); return;
    case T::Num: out->append(n->s.data(), n->s.size()); return;
    case T::Str: put_string(out, n->s); return;
    default: break;
  }
  if (!n->enc.empty()) {
    out->append(n->enc.data(), n->enc.size());
    return;
  }
  if (depth < cache_depth) {  // encode into the node's own buffer, then splice it in
    n->enc.reserve(n->hint ? n->hint + 64 : (depth == 0 ? 1024 : 128));
    write_body(&n->enc, n, depth, cache_depth);
    out->append(n->enc.data(), n->enc.size());
    return;
  }
  write_body(out, n, depth, cache_depth);
}

// the node's bytes, encoded (and cached) on first use: a stored object's reply and watch events
inline const jstr& encoded(Node* n) {
  if (n->enc.empty() && (n->t == T::Obj || n->t == T::Arr)) {
    n->enc.reserve(n->hint ? n->hint + 64 : 1024);
    write_body(&n->enc, n, 0, 2);
  }
  return n->enc;
}

inline std::string dump(Node* n, int cache_depth = 2) {
  std::string out;
  write(&out, n, 0, cache_depth);
  return out;
}

// ------------------------------------------------------------------ compare / merge

inline bool num_equal(const jstr& a, const jstr& b) {
  if (a == b) return true;
  return std::strtod(a.c_str(), nullptr) == std::strtod(b.c_str(), nullptr);
}

// Python's `==` on decoded JSON (1 == 1.0, key order ignored)
inline bool equal(const Node* a, const Node* b) {
  if (a == b) return true;
  if (!a || !b) return false;
  if (a->t != b->t) return false;
  switch (a->t) {
    case T::Null:
    case T::True:
    case T::False: return true;
    case T::Num: return num_equal(a->s, b->s);
    case T::Str: return a->s == b->s;
    case T::Arr:
      if (a->a.size() != b->a.size()) return false;
      for (size_t i = 0; i < a->a.size(); ++i)
        if (!equal(a->a[i].get(), b->a[i].get())) return false;
      return true;
    case T::Obj: {
      if (a->o.size() != b->o.size()) return false;
      for (size_t i = 0; i < a->o.size(); ++i) {
        const Member& m = a->o[i];
        // same key order (the common case) first, then a lookup
        const Ref* bv = (b->o[i].first == m.first) ? &b->o[i].second : b->get(std::string_view(m.first));
        if (!bv || !equal(m.second.get(), bv->get())) return false;
      }
      return true;
    }
  }
  return false;
}

// RFC 7386 JSON merge patch; untouched members of `target` are shared, not copied
inline Ref merge_patch(const Ref& target, const Ref& patch) {
  if (!patch->is_obj()) return patch;
  Ref out = (target && target->is_obj()) ? shallow(target.get()) : mk_obj();
  Node* o = out.get();
  for (const Member& m : patch->o) {
    if (m.second->t == T::Null) {
      for (size_t i = 0; i < o->o.size(); ++i)
        if (o->o[i].first == m.first) {
          o->o.erase(o->o.begin() + static_cast<long>(i));
          break;
        }
      continue;
    }
    const Ref* cur = o->get(std::string_view(m.first));
    Ref merged = merge_patch(cur ? *cur : Ref(), m.second);
    if (cur) {
      for (auto& mm : o->o)
        if (mm.first == m.first) {
          mm.second = std::move(merged);
          break;
        }
    } else {
      o->o.emplace_back(m.first, std::move(merged));
    }
  }
  return out;
}

// deep copy (a private tree: e.g. a schema default inserted into a fresh object)
inline Ref deep_copy(const Node* n) {
  Node* c = new Node(n->t);
  c->s = n->s;
  c->a.reserve(n->a.size());
  for (const Ref& v : n->a) c->a.push_back(deep_copy(v.get()));
  c->o.reserve(n->o.size());
  for (const Member& m : n->o) c->o.emplace_back(m.first, deep_copy(m.second.get()));
  return Ref(c);
}

// mark a stored tree admitted (stops at subtrees already marked: they are shared, old)
inline void mark_admitted(Node* n) {
  if (n->admitted) return;
  n->admitted = true;
  for (const Ref& v : n->a) mark_admitted(v.get());
  for (const Member& m : n->o) mark_admitted(m.second.get());
}

}  // namespace jdom
