// Native HTTP/1.1 message framing (CPython extension `_httpcodec`).
//
// Every API call the operator makes is one HTTP/1.1 exchange with the
// apiserver (reference: client-go REST over net/http), and the
// fake apiserver's front end parses every one of them again on the other side.
// In the 1000-Cron bench the Python head parsers were the largest single item
// of the fake apiserver's request path (~10% of its CPU) and a visible one of
// the operator's.  These two functions do the framing in one pass over the
// receive buffer and hand back ready Python objects:
//
//   parse_request(buf, max_body) -> None | int | tuple
//       None   the request is incomplete
//       100    incomplete, and it carries "Expect: 100-continue"
//       400    malformed request line or framing (bad Content-Length / chunk size)
//       413    Content-Length above max_body
//       431    no end of head within 1 MiB
//       (method, target, headers, body, consumed, keep_alive)
//           headers: lower-cased, stripped keys -> stripped values (latin-1, last
//           duplicate wins); body: bytes, de-chunked; consumed: bytes of buf used
//
//   parse_response(buf) -> None | -1 | tuple
//       None   the response is incomplete
//       -1     not framed by Content-Length/chunked, or an interim 1xx: the caller's
//              incremental parser handles it
//       (status, body, consumed, close, retry_after)
//           retry_after: int seconds for status >= 400 with a numeric Retry-After,
//           else None
//
// Semantics mirror the pure-Python parsers they replace (apiserver/http.py
// _ServerConn._next_request, runtime/fasthttp.py _Conn._parse), which remain
// the fallback and the oracle of tests/test_httpcodec.py.

#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include <cstdint>
#include <cstring>

#include "httpframe.h"

namespace {

using namespace httpframe;

constexpr Py_ssize_t kMaxHead = 1 << 20;

PyObject* latin1(const unsigned char* b, const unsigned char* e) {
  return PyUnicode_DecodeLatin1(reinterpret_cast<const char*>(b), e - b, nullptr);
}

// lower-cased latin-1 key; non-ASCII letters go through str.lower() like the Python parser
PyObject* lower_key(const unsigned char* b, const unsigned char* e) {
  bool ascii = true;
  for (const unsigned char* p = b; p < e; ++p)
    if (*p >= 0x80) {
      ascii = false;
      break;
    }
  if (!ascii) {
    PyObject* s = latin1(b, e);
    if (!s) return nullptr;
    PyObject* r = PyObject_CallMethod(s, "lower", nullptr);
    Py_DECREF(s);
    return r;
  }
  PyObject* s = PyUnicode_New(e - b, 127);
  if (!s) return nullptr;
  Py_UCS1* d = PyUnicode_1BYTE_DATA(s);
  for (const unsigned char* p = b; p < e; ++p) *d++ = lower(*p);
  return s;
}

struct Buf {
  Py_buffer view{};
  bool ok = false;
  explicit Buf(PyObject* o) { ok = PyObject_GetBuffer(o, &view, PyBUF_SIMPLE) == 0; }
  ~Buf() {
    if (ok) PyBuffer_Release(&view);
  }
  const unsigned char* begin() const { return static_cast<const unsigned char*>(view.buf); }
  const unsigned char* end() const { return begin() + view.len; }
};

// Chunked body starting at p: 0 = incomplete, -1 = malformed, else bytes consumed from p.
// Body bytes are appended to *body (created on first use).
Py_ssize_t dechunk(const unsigned char* p0, const unsigned char* e, PyObject** body) {
  const unsigned char* p = p0;
  // two passes: measure, then copy once
  Py_ssize_t total = 0;
  const unsigned char* q = p;
  Py_ssize_t consumed = 0;
  for (;;) {
    const unsigned char* nl = find(q, e, "\r\n", 2);
    if (!nl) return 0;
    const unsigned char* semi = static_cast<const unsigned char*>(memchr(q, ';', static_cast<size_t>(nl - q)));
    long long size;
    if (!parse_hex(q, semi ? semi : nl, &size)) return -1;
    if (size == 0) {
      // trailers end with an empty line; the search starts at this line's CRLF
      const unsigned char* tend = find(nl, e, "\r\n\r\n", 4);
      if (!tend) return 0;
      consumed = (tend + 4) - p0;
      break;
    }
    if (e - (nl + 2) < size + 2) return 0;
    total += static_cast<Py_ssize_t>(size);
    q = nl + 2 + size + 2;
  }
  PyObject* out = PyBytes_FromStringAndSize(nullptr, total);
  if (!out) return -2;
  char* d = PyBytes_AS_STRING(out);
  q = p;
  for (;;) {
    const unsigned char* nl = find(q, e, "\r\n", 2);
    const unsigned char* semi = static_cast<const unsigned char*>(memchr(q, ';', static_cast<size_t>(nl - q)));
    long long size;
    parse_hex(q, semi ? semi : nl, &size);
    if (size == 0) break;
    std::memcpy(d, nl + 2, static_cast<size_t>(size));
    d += size;
    q = nl + 2 + size + 2;
  }
  *body = out;
  return consumed;
}

PyObject* parse_request(PyObject*, PyObject* args) {
  PyObject* obj;
  Py_ssize_t max_body;
  if (!PyArg_ParseTuple(args, "On", &obj, &max_body)) return nullptr;
  Buf buf(obj);
  if (!buf.ok) return nullptr;
  const unsigned char* b = buf.begin();
  const unsigned char* e = buf.end();
  const unsigned char* hend = find(b, e, "\r\n\r\n", 4);
  if (!hend) {
    if (e - b > kMaxHead) return PyLong_FromLong(431);
    Py_RETURN_NONE;
  }
  // request line: METHOD SP TARGET SP VERSION
  const unsigned char* l_end = find(b, hend + 2, "\r\n", 2);
  const unsigned char* sp1 = static_cast<const unsigned char*>(memchr(b, ' ', static_cast<size_t>(l_end - b)));
  if (!sp1) return PyLong_FromLong(400);
  const unsigned char* sp2 =
      static_cast<const unsigned char*>(memchr(sp1 + 1, ' ', static_cast<size_t>(l_end - sp1 - 1)));
  if (!sp2) return PyLong_FromLong(400);
  const unsigned char* ver_b = sp2 + 1;
  const bool http11 = (l_end - ver_b) == 8 && std::memcmp(ver_b, "HTTP/1.1", 8) == 0;

  PyObject* headers = PyDict_New();
  if (!headers) return nullptr;
  long long clen = 0;
  bool have_clen = false, clen_bad = false, chunked = false, expect_continue = false;
  int conn = 0;  // 0 none/other, 1 close, 2 keep-alive
  const unsigned char* p = l_end + 2;
  while (p < hend + 2) {
    const unsigned char* nl = find(p, hend + 2, "\r\n", 2);
    const unsigned char* colon = static_cast<const unsigned char*>(memchr(p, ':', static_cast<size_t>(nl - p)));
    const unsigned char *kb = p, *ke = colon ? colon : nl;
    const unsigned char *vb = colon ? colon + 1 : nl, *ve = nl;
    strip(kb, ke);
    strip(vb, ve);
    PyObject* k = lower_key(kb, ke);
    PyObject* v = k ? latin1(vb, ve) : nullptr;
    if (!v || PyDict_SetItem(headers, k, v) < 0) {
      Py_XDECREF(k);
      Py_XDECREF(v);
      Py_DECREF(headers);
      return nullptr;
    }
    Py_DECREF(k);
    Py_DECREF(v);
    // framing headers (last occurrence wins, like the dict)
    if (ieq(kb, ke, "content-length")) {
      have_clen = vb != ve;
      clen_bad = have_clen && !parse_dec(vb, ve, &clen);
      if (!have_clen) clen = 0;
    } else if (ieq(kb, ke, "transfer-encoding")) {
      chunked = icontains(vb, ve, "chunked");
    } else if (ieq(kb, ke, "expect")) {
      expect_continue = ieq(vb, ve, "100-continue");
    } else if (ieq(kb, ke, "connection")) {
      conn = ieq(vb, ve, "close") ? 1 : ieq(vb, ve, "keep-alive") ? 2 : 0;
    }
    p = nl + 2;
  }
  const unsigned char* body_b = hend + 4;
  PyObject* body = nullptr;
  Py_ssize_t consumed;
  if (chunked) {
    Py_ssize_t n = dechunk(body_b, e, &body);
    if (n == 0) {
      Py_DECREF(headers);
      Py_RETURN_NONE;
    }
    if (n < 0) {
      Py_DECREF(headers);
      if (n == -2) return nullptr;
      return PyLong_FromLong(400);
    }
    consumed = (body_b - b) + n;
  } else {
    if (clen_bad) {
      Py_DECREF(headers);
      return PyLong_FromLong(400);
    }
    if (clen > max_body) {
      Py_DECREF(headers);
      return PyLong_FromLong(413);
    }
    if (e - body_b < clen) {
      Py_DECREF(headers);
      if (expect_continue) return PyLong_FromLong(100);
      Py_RETURN_NONE;
    }
    body = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(body_b), static_cast<Py_ssize_t>(clen));
    if (!body) {
      Py_DECREF(headers);
      return nullptr;
    }
    consumed = (body_b - b) + static_cast<Py_ssize_t>(clen);
  }
  const bool keep = http11 ? conn != 1 : conn == 2;
  PyObject* method = latin1(b, sp1);
  PyObject* target = method ? latin1(sp1 + 1, sp2) : nullptr;
  if (!target) {
    Py_XDECREF(method);
    Py_DECREF(headers);
    Py_DECREF(body);
    return nullptr;
  }
  // (method, target, headers, body, consumed, keep_alive); N steals the references
  return Py_BuildValue("(NNNNnO)", method, target, headers, body, consumed, keep ? Py_True : Py_False);
}

PyObject* parse_response(PyObject*, PyObject* args) {
  PyObject* obj;
  if (!PyArg_ParseTuple(args, "O", &obj)) return nullptr;
  Buf buf(obj);
  if (!buf.ok) return nullptr;
  const unsigned char* b = buf.begin();
  const unsigned char* e = buf.end();
  const unsigned char* hend = find(b, e, "\r\n\r\n", 4);
  if (!hend) Py_RETURN_NONE;
  ResponseHead h;
  if (!parse_response_head(b, hend, &h)) return PyLong_FromLong(-1);
  const long long status = h.status;
  if (status >= 100 && status < 200) return PyLong_FromLong(-1);  // interim: incremental parser
  const bool close = h.close, chunked = h.chunked;
  const long long clen = h.content_length, retry_after = h.retry_after;
  const unsigned char* body_b = hend + 4;
  PyObject* body = nullptr;
  Py_ssize_t consumed;
  if (status == 204 || status == 304) {
    body = PyBytes_FromStringAndSize("", 0);
    consumed = body_b - b;
  } else if (chunked) {
    Py_ssize_t n = dechunk(body_b, e, &body);
    if (n == 0) Py_RETURN_NONE;
    if (n == -2) return nullptr;
    if (n < 0) return PyLong_FromLong(-1);
    consumed = (body_b - b) + n;
  } else if (clen >= 0) {
    if (e - body_b < clen) Py_RETURN_NONE;
    body = PyBytes_FromStringAndSize(reinterpret_cast<const char*>(body_b), static_cast<Py_ssize_t>(clen));
    consumed = (body_b - b) + static_cast<Py_ssize_t>(clen);
  } else {
    return PyLong_FromLong(-1);  // read until close
  }
  if (!body) return nullptr;
  PyObject* ra;
  if (status >= 400 && retry_after >= 0) {
    ra = PyLong_FromLongLong(retry_after);
    if (!ra) {
      Py_DECREF(body);
      return nullptr;
    }
  } else {
    Py_INCREF(Py_None);
    ra = Py_None;
  }
  return Py_BuildValue("(LNnON)", status, body, consumed, close ? Py_True : Py_False, ra);
}

PyMethodDef kMethods[] = {
    {"parse_request", parse_request, METH_VARARGS,
     "parse_request(buf, max_body) -> None | int | (method, target, headers, body, consumed, keep_alive)"},
    {"parse_response", parse_response, METH_VARARGS,
     "parse_response(buf) -> None | -1 | (status, body, consumed, close, retry_after)"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_httpcodec", "Native HTTP/1.1 message framing.", -1, kMethods,
                       nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__httpcodec(void) { return PyModule_Create(&kModule); }
