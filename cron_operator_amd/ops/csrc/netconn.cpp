// Native HTTP/1.1 client connection for the asyncio event loop (CPython extension `_netconn`).
//
// Every API call the operator makes is one HTTP/1.1 exchange with the apiserver and every
// cache update arrives on a watch stream (reference: client-go REST + watch over net/http,
// used by controller-runtime's client and informers -- /root/reference/cmd/operator/start.go
// builds that rest config).  Profiling one operator process at 1000 Crons put
// the Python side of that plumbing -- asyncio's selector transport, the protocol callbacks,
// response framing and de-chunking, TLS through asyncio's pure-Python SSL protocol -- at a
// tenth of the process's CPU.  `Conn` does the same work in one object that the loop calls
// directly:
//
//   * the socket (already connected by the caller, handed over as a file descriptor) is
//     registered with the loop once (`loop.add_reader(fd, conn._on_readable)`); a readiness
//     callback receives, frames and completes the in-flight response in C++;
//   * TLS is OpenSSL on the socket itself (non-blocking `SSL_connect`/`SSL_read`/`SSL_write`),
//     configured by a `TlsContext`: an `SSL_CTX` this extension builds from the kubeconfig's
//     PEM material (CA, client certificate and key, verify mode, ALPN) with the libssl it is
//     linked against.  Hostname checks and SNI follow what
//     `SSLContext.wrap_socket(server_hostname=...)` does.  A plain `ssl.SSLContext` is accepted
//     only when CPython's `_ssl` module is provably linked to that same libssl (configure()
//     checks the version and that `_ssl`'s `SSL_CTX_new` is ours); otherwise the caller keeps
//     asyncio's TLS transports -- its `SSL_CTX` is never touched;
//   * request mode: `send(data) -> Future[(status, body, retry_after)]`, Content-Length,
//     chunked and read-until-close bodies, interim 1xx responses skipped, keep-alive;
//   * stream mode (`open_stream(data, decode) -> Future[status]`): the body of a watch is
//     de-chunked and split into lines; each non-empty line is decoded by `decode` (a native
//     `_fastjson.Codec` in the operator) and queued; `take()` hands over the whole batch and
//     `wait()` returns a future that completes when items arrive or the stream ends.
//
// Failure semantics are those of the Python protocols in runtime/fasthttp.py (`_Conn`,
// `_StreamConn`), which stay the fallback (proxies, or no native build) and the oracle of
// tests/test_netconn.py: a connection lost before the response raises
// `ConnectionFailed(msg, no_response, reused)` so the pool can retry a stale keep-alive
// connection once; an error status on a stream raises `HttpStatusError(status, body)`.
//
// Everything runs on the loop's thread under the GIL; nothing here blocks.

#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <structmember.h>

#include <arpa/inet.h>
#include <dlfcn.h>
#include <errno.h>
#include <openssl/crypto.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "httpframe.h"

namespace {

using namespace httpframe;

constexpr size_t kMaxHead = 1 << 20;
constexpr size_t kReadChunk = 256 * 1024;
constexpr size_t kMaxReadPerWake = 4 << 20;  // bound one callback's work on a busy stream

// exception classes installed by configure(): ConnectionFailed(msg, no_response, reused),
// HttpStatusError(status, body), ssl.SSLError(msg)
PyObject* g_conn_failed = nullptr;
PyObject* g_status_error = nullptr;
PyObject* g_ssl_error = nullptr;

PyObject *s_create_future, *s_set_result, *s_set_exception, *s_done, *s_add_reader, *s_remove_reader,
    *s_add_writer, *s_remove_writer, *s_on_readable, *s_on_writable, *s_options, *s_verify_mode;

// one receive buffer for every connection: all callbacks run on the loop's thread under the GIL
char g_rbuf[kReadChunk];

enum Mode { kRequest = 0, kStream = 1 };
enum Handshake { kHsNone = 0, kHsRunning = 1 };
enum IoResult : long { kWantRead = -1, kWantWrite = -2, kIoError = -3 };

// parser states (request mode): head, Content-Length body, chunked body, body until close
enum RespState { kHead = 0, kLength = 1, kChunked = 2, kUntilClose = 3 };

struct Core {
  std::string rbuf;  // received, not yet consumed: rbuf[rpos:]
  size_t rpos = 0;
  std::string wbuf;  // request bytes not written yet: wbuf[wpos:]
  size_t wpos = 0;
  // request mode: the response being parsed
  int state = kHead;
  long long status = 0, clen = -1, retry_after = -1;
  bool close_after = false;
  std::string body;
  // stream mode
  long long sstatus = 0, sclen = -1;
  bool schunked = false;
  std::string lines;
  std::string err_body;
};

struct ConnObject {
  PyObject_HEAD
  Core* core;
  PyObject* loop;
  PyObject* ssl_ctx;   // the TlsContext / ssl.SSLContext (keeps its SSL_CTX alive)
  SSL* ssl;
  int fd;
  int mode;
  int hs;
  PyObject* hs_fut;    // TLS handshake
  PyObject* fut;       // request mode: the response; stream mode: the head (status)
  PyObject* decode;    // stream mode: bytes line -> item
  PyObject* items;     // stream mode: decoded items not taken yet (list)
  PyObject* waiter;    // stream mode: wait() future
  PyObject* stream_error;
  PyObject* weakrefs;
  PyObject* pool;      // the Pool whose request is in flight here (strong; set only while busy)
  long used;           // requests sent on this connection
  long ssl_gen;        // pool bookkeeping (TLS context generation)
  double deadline;     // pool bookkeeping (loop time the in-flight response is due by)
  bool alive;
  bool got_any;        // a byte of the in-flight response arrived
  bool reader_on;
  bool writer_on;
  bool stream_done;
};

// A keep-alive pool of request-mode connections to one server (`_netconn.Pool`): the request
// path of runtime/fasthttp.py's HttpPool -- build the request head, take an idle connection,
// send, and give the connection back when its response completes -- without a Python frame.
struct PoolObject {
  PyObject_HEAD
  std::vector<ConnObject*>* idle;  // strong references; the most recently used at the back
  std::vector<ConnObject*>* busy;  // strong references; each has `pool` set to this pool
  std::string* target;             // request-target prefix (base path, or absolute form via a proxy)
  std::string* fixed;              // header lines sent with every request (Host, auth, ...)
  Py_ssize_t max_idle;
  double timeout;                  // seconds a response may take (deadline sweep)
  long ssl_gen;                    // connections of another TLS generation are not reused
  bool closed;
  PyObject* weakrefs;
};

PyObject* g_timeout_error = nullptr;  // asyncio.TimeoutError, for the deadline sweep
// configure(): CPython's _ssl module runs on this extension's libssl (same build, same symbols)
bool g_shared_openssl = false;

// The exchange on `s` ended (response completed or connection lost): leave the pool's busy
// list, and go back to the idle list when reusable (closed otherwise).  May drop the last
// reference to `s`: callers hold their own.
void pool_release(ConnObject* s);

// ----------------------------------------------------------------------------- helpers

// fut.set_result(value) unless fut is done (cancelled, or failed by a deadline sweep); steals nothing
void resolve(PyObject* fut, PyObject* value) {
  if (!fut) return;
  PyObject* d = PyObject_CallMethodNoArgs(fut, s_done);
  if (!d) {
    PyErr_Clear();
    return;
  }
  const bool done = d == Py_True;
  Py_DECREF(d);
  if (done) return;
  PyObject* r = PyObject_CallMethodOneArg(fut, s_set_result, value);
  if (!r) PyErr_Clear();
  Py_XDECREF(r);
}

void reject(PyObject* fut, PyObject* exc) {
  if (!fut || !exc) {
    PyErr_Clear();
    return;
  }
  PyObject* d = PyObject_CallMethodNoArgs(fut, s_done);
  if (!d) {
    PyErr_Clear();
    return;
  }
  const bool done = d == Py_True;
  Py_DECREF(d);
  if (done) return;
  PyObject* r = PyObject_CallMethodOneArg(fut, s_set_exception, exc);
  if (!r) PyErr_Clear();
  Py_XDECREF(r);
}

PyObject* conn_failed(const std::string& msg, bool no_response, bool reused) {
  return PyObject_CallFunction(g_conn_failed, "s#OO", msg.data(), static_cast<Py_ssize_t>(msg.size()),
                               no_response ? Py_True : Py_False, reused ? Py_True : Py_False);
}

PyObject* status_error(long long status, const std::string& body) {
  return PyObject_CallFunction(g_status_error, "Ly#", status, body.data(), static_cast<Py_ssize_t>(body.size()));
}

PyObject* ssl_error(const std::string& msg) {
  return PyObject_CallFunction(g_ssl_error, "s#", msg.data(), static_cast<Py_ssize_t>(msg.size()));
}

std::string ssl_error_string(SSL* ssl, int err) {
  std::string msg;
  char buf[256];
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    ERR_error_string_n(e, buf, sizeof buf);
    if (!msg.empty()) msg += "; ";
    msg += buf;
  }
  if (ssl) {
    const long vr = SSL_get_verify_result(ssl);
    if (vr != X509_V_OK) {
      msg += msg.empty() ? "" : " ";
      msg += "(certificate verify failed: ";
      msg += X509_verify_cert_error_string(vr);
      msg += ")";
    }
  }
  if (msg.empty()) {
    if (err == SSL_ERROR_SYSCALL) msg = errno ? std::strerror(errno) : "unexpected EOF in TLS";
    else msg = "TLS error " + std::to_string(err);
  }
  return msg;
}

void set_reader(ConnObject* s, bool on) {
  if (s->fd < 0 || !s->loop || s->reader_on == on) return;
  PyObject* r;
  PyObject* fd = PyLong_FromLong(s->fd);
  if (!fd) {
    PyErr_Clear();
    return;
  }
  if (on) {
    PyObject* cb = PyObject_GetAttr(reinterpret_cast<PyObject*>(s), s_on_readable);
    r = cb ? PyObject_CallMethodObjArgs(s->loop, s_add_reader, fd, cb, nullptr) : nullptr;
    Py_XDECREF(cb);
  } else {
    r = PyObject_CallMethodObjArgs(s->loop, s_remove_reader, fd, nullptr);
  }
  Py_DECREF(fd);
  if (r) s->reader_on = on;
  else PyErr_Clear();  // a closed loop: nothing is registered any more
  Py_XDECREF(r);
}

void set_writer(ConnObject* s, bool on) {
  if (s->fd < 0 || !s->loop || s->writer_on == on) return;
  PyObject* r;
  PyObject* fd = PyLong_FromLong(s->fd);
  if (!fd) {
    PyErr_Clear();
    return;
  }
  if (on) {
    PyObject* cb = PyObject_GetAttr(reinterpret_cast<PyObject*>(s), s_on_writable);
    r = cb ? PyObject_CallMethodObjArgs(s->loop, s_add_writer, fd, cb, nullptr) : nullptr;
    Py_XDECREF(cb);
  } else {
    r = PyObject_CallMethodObjArgs(s->loop, s_remove_writer, fd, nullptr);
  }
  Py_DECREF(fd);
  if (r) s->writer_on = on;
  else PyErr_Clear();
  Py_XDECREF(r);
}

// Unregister and close the socket (and the TLS session).  Futures are left to the caller.
void close_io(ConnObject* s) {
  s->alive = false;
  if (s->fd < 0) return;
  set_reader(s, false);
  set_writer(s, false);
  if (s->ssl) {
    SSL_free(s->ssl);
    s->ssl = nullptr;
  }
  ::close(s->fd);
  s->fd = -1;
}

// >0 bytes, 0 EOF, kWantRead, kWantWrite, kIoError (*err set)
long io_read(ConnObject* s, char* buf, size_t n, std::string* err) {
  if (!s->ssl) {
    for (;;) {
      const ssize_t r = ::recv(s->fd, buf, n, 0);
      if (r >= 0) return static_cast<long>(r);
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) return kWantRead;
      *err = std::strerror(errno);
      return kIoError;
    }
  }
  ERR_clear_error();
  errno = 0;
  const int r = SSL_read(s->ssl, buf, static_cast<int>(n));
  if (r > 0) return r;
  const int e = SSL_get_error(s->ssl, r);
  switch (e) {
    case SSL_ERROR_WANT_READ: return kWantRead;
    case SSL_ERROR_WANT_WRITE: return kWantWrite;
    case SSL_ERROR_ZERO_RETURN: return 0;
    case SSL_ERROR_SYSCALL:
      if (ERR_peek_error() == 0 && errno == 0) return 0;  // EOF without close_notify
      if (errno == EAGAIN || errno == EWOULDBLOCK) return kWantRead;
      [[fallthrough]];
    default:
      *err = ssl_error_string(s->ssl, e);
      return kIoError;
  }
}

long io_write(ConnObject* s, const char* buf, size_t n, std::string* err) {
  if (!s->ssl) {
    for (;;) {
      const ssize_t r = ::send(s->fd, buf, n, MSG_NOSIGNAL);
      if (r >= 0) return static_cast<long>(r);
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) return kWantWrite;
      *err = std::strerror(errno);
      return kIoError;
    }
  }
  ERR_clear_error();
  errno = 0;
  const int r = SSL_write(s->ssl, buf, static_cast<int>(n));
  if (r > 0) return r;
  const int e = SSL_get_error(s->ssl, r);
  switch (e) {
    case SSL_ERROR_WANT_READ: return kWantRead;
    case SSL_ERROR_WANT_WRITE: return kWantWrite;
    case SSL_ERROR_SYSCALL:
      if (errno == EAGAIN || errno == EWOULDBLOCK) return kWantWrite;
      [[fallthrough]];
    default:
      *err = ssl_error_string(s->ssl, e);
      return kIoError;
  }
}

// ----------------------------------------------------------------------------- connection loss

// The connection broke or the peer closed it (`connection_lost` of the Python protocols).
void lost(ConnObject* s, const std::string& why);

// ----------------------------------------------------------------------------- request mode

void reset_response(Core& c) {
  c.state = kHead;
  c.status = 0;
  c.clen = -1;
  c.retry_after = -1;
  c.close_after = false;
  c.body.clear();
}

// Complete the in-flight response with the parsed status and body [b, b + n).
void finish_response(ConnObject* s, const char* b, size_t n) {
  Core& c = *s->core;
  PyObject* body = PyBytes_FromStringAndSize(b, static_cast<Py_ssize_t>(n));
  PyObject* ra;
  if (c.status >= 400 && c.retry_after >= 0) ra = PyLong_FromLongLong(c.retry_after);
  else {
    Py_INCREF(Py_None);
    ra = Py_None;
  }
  PyObject* result = (body && ra) ? Py_BuildValue("(LNN)", c.status, body, ra) : nullptr;
  if (!result) {
    Py_XDECREF(body);
    Py_XDECREF(ra);
    PyErr_Clear();
  }
  // a response that overtook the rest of its request (an early error status): the unsent
  // bytes would precede the next request on the wire, so this connection is not reused
  const bool close_after = c.close_after || c.wpos < c.wbuf.size();
  reset_response(c);
  if (close_after) close_io(s);
  PyObject* fut = s->fut;
  s->fut = nullptr;
  pool_release(s);  // idle again before the caller resumes
  if (result) resolve(fut, result);
  else {
    PyObject* exc = conn_failed("out of memory decoding the response", false, false);
    reject(fut, exc);
    Py_XDECREF(exc);
  }
  Py_XDECREF(result);
  Py_XDECREF(fut);
}

// Advance the response parser over rbuf[rpos:].  1: a response completed (and was delivered),
// 0: more bytes needed, -1: malformed (the caller drops the connection).
int parse_response(ConnObject* s) {
  Core& c = *s->core;
  for (;;) {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rpos;
    const unsigned char* e = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rbuf.size();
    if (c.state == kHead) {
      const unsigned char* hend = find(b, e, "\r\n\r\n", 4);
      if (!hend) return static_cast<size_t>(e - b) > kMaxHead ? -1 : 0;
      ResponseHead h;
      if (!parse_response_head(b, hend, &h)) return -1;
      c.rpos += static_cast<size_t>(hend + 4 - b);
      c.status = h.status;
      c.close_after = h.close;
      c.retry_after = h.retry_after;
      if (h.status >= 100 && h.status < 200) continue;  // interim response: the next head follows
      if (h.status == 204 || h.status == 304) {
        finish_response(s, "", 0);
        return 1;
      }
      if (h.chunked) {
        c.state = kChunked;
        c.body.clear();
      } else if (h.content_length >= 0) {
        c.state = kLength;
        c.clen = h.content_length;
      } else {
        c.state = kUntilClose;
        c.close_after = true;
      }
      continue;
    }
    if (c.state == kLength) {
      if (e - b < c.clen) return 0;
      const size_t n = static_cast<size_t>(c.clen);
      const size_t at = c.rpos;
      c.rpos += n;
      // deliver straight from the receive buffer: finishing may close the socket, never the buffer
      finish_response(s, c.rbuf.data() + at, n);
      if (c.rpos == c.rbuf.size()) {
        c.rbuf.clear();  // keeps its capacity for the next response
        c.rpos = 0;
      }
      return 1;
    }
    if (c.state == kChunked) {
      for (;;) {
        b = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rpos;
        const unsigned char* nl = find(b, e, "\r\n", 2);
        if (!nl) return 0;
        long long size;
        if (!chunk_size(b, nl, &size)) return -1;
        if (size == 0) {
          // trailers end with an empty line; the search starts at this line's CRLF
          const unsigned char* tend = find(nl, e, "\r\n\r\n", 4);
          if (!tend) return 0;
          c.rpos += static_cast<size_t>(tend + 4 - b);
          std::string body;
          body.swap(c.body);
          c.rbuf.erase(0, c.rpos);
          c.rpos = 0;
          finish_response(s, body.data(), body.size());
          return 1;
        }
        if (e - (nl + 2) < size + 2) return 0;
        c.body.append(reinterpret_cast<const char*>(nl + 2), static_cast<size_t>(size));
        c.rpos += static_cast<size_t>(nl + 2 + size + 2 - b);
      }
    }
    // kUntilClose: everything is body; the response completes at EOF
    c.body.append(reinterpret_cast<const char*>(b), static_cast<size_t>(e - b));
    c.rbuf.clear();
    c.rpos = 0;
    return 0;
  }
}

// ----------------------------------------------------------------------------- stream mode

void wake(ConnObject* s) {
  if (s->waiter) {
    PyObject* w = s->waiter;
    s->waiter = nullptr;
    resolve(w, Py_None);
    Py_DECREF(w);
  }
}

// The body bytes received so far, de-chunked when chunked, appended to *out.
void stream_body(ConnObject* s, std::string* out) {
  Core& c = *s->core;
  if (!c.schunked) {
    out->append(c.rbuf, c.rpos, std::string::npos);
    c.rbuf.clear();
    c.rpos = 0;
    return;
  }
  for (;;) {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rpos;
    const unsigned char* e = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rbuf.size();
    const unsigned char* nl = find(b, e, "\r\n", 2);
    if (!nl) break;
    long long size;
    if (!chunk_size(b, nl, &size)) {
      s->stream_done = true;  // malformed framing: end the stream
      c.rbuf.clear();
      c.rpos = 0;
      break;
    }
    if (size == 0) {
      s->stream_done = true;
      c.rbuf.clear();
      c.rpos = 0;
      break;
    }
    if (e - (nl + 2) < size + 2) break;
    out->append(reinterpret_cast<const char*>(nl + 2), static_cast<size_t>(size));
    c.rpos += static_cast<size_t>(nl + 2 + size + 2 - b);
  }
  if (c.rpos > 0 && c.rpos == c.rbuf.size()) {
    c.rbuf.clear();
    c.rpos = 0;
  } else if (c.rpos > (1 << 16)) {
    c.rbuf.erase(0, c.rpos);
    c.rpos = 0;
  }
}

void fail_stream_head(ConnObject* s, PyObject* exc) {
  PyObject* h = s->fut;
  s->fut = nullptr;
  reject(h, exc);
  Py_XDECREF(h);
}

// Decode complete lines into items.  false: the decoder raised (the stream ends with that error).
bool stream_lines(ConnObject* s) {
  Core& c = *s->core;
  bool got = false;
  size_t pos = 0;
  for (;;) {
    const size_t nl = c.lines.find('\n', pos);
    if (nl == std::string::npos) break;
    size_t b = pos, e = nl;
    pos = nl + 1;
    while (b < e && is_bytes_space(static_cast<unsigned char>(c.lines[b]))) ++b;
    while (e > b && is_bytes_space(static_cast<unsigned char>(c.lines[e - 1]))) --e;
    if (b == e) continue;
    PyObject* line = PyBytes_FromStringAndSize(c.lines.data() + b, static_cast<Py_ssize_t>(e - b));
    PyObject* item = line ? PyObject_CallOneArg(s->decode, line) : nullptr;
    Py_XDECREF(line);
    if (!item || PyList_Append(s->items, item) < 0) {
      Py_XDECREF(item);
      PyObject *type, *value, *tb;
      PyErr_Fetch(&type, &value, &tb);
      PyErr_NormalizeException(&type, &value, &tb);
      Py_XDECREF(type);
      Py_XDECREF(tb);
      Py_XSETREF(s->stream_error, value);
      c.lines.erase(0, pos);
      if (got) wake(s);
      return false;
    }
    Py_DECREF(item);
    got = true;
  }
  c.lines.erase(0, pos);
  if (got) wake(s);
  return true;
}

// 0: keep going, -1: the stream ended (malformed head or decode error; the caller closes)
int parse_stream(ConnObject* s) {
  Core& c = *s->core;
  if (c.sstatus == 0) {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rpos;
    const unsigned char* e = reinterpret_cast<const unsigned char*>(c.rbuf.data()) + c.rbuf.size();
    const unsigned char* hend = find(b, e, "\r\n\r\n", 4);
    if (!hend) {
      if (static_cast<size_t>(e - b) <= kMaxHead) return 0;
      PyObject* exc = conn_failed("stream response head too large", false, false);
      fail_stream_head(s, exc);
      Py_XDECREF(exc);
      return -1;
    }
    ResponseHead h;
    if (!parse_response_head(b, hend, &h) || h.status <= 0) {
      PyObject* exc = conn_failed("bad HTTP response head on a stream", false, false);
      fail_stream_head(s, exc);
      Py_XDECREF(exc);
      return -1;
    }
    c.rpos += static_cast<size_t>(hend + 4 - b);
    c.sstatus = h.status;
    c.schunked = h.chunked;
    c.sclen = h.content_length;
    if (h.status < 400) {
      PyObject* st = PyLong_FromLongLong(h.status);
      PyObject* f = s->fut;
      s->fut = nullptr;
      if (st) resolve(f, st);
      else PyErr_Clear();
      Py_XDECREF(st);
      Py_XDECREF(f);
    }
  }
  if (c.sstatus >= 400) {  // collect the error body, then fail the open
    stream_body(s, &c.err_body);
    if ((c.sclen >= 0 && static_cast<long long>(c.err_body.size()) >= c.sclen) || s->stream_done) {
      PyObject* exc = status_error(c.sstatus, c.err_body);
      fail_stream_head(s, exc);
      Py_XDECREF(exc);
    }
    return 0;
  }
  stream_body(s, &c.lines);
  if (!stream_lines(s)) {
    s->stream_done = true;
    return -1;
  }
  if (s->stream_done) wake(s);
  return 0;
}

// ----------------------------------------------------------------------------- loss / reads / writes

void lost(ConnObject* s, const std::string& why) {
  Core& c = *s->core;
  if (s->mode == kStream) {
    s->stream_done = true;
    if (s->fut) {  // the head never completed
      PyObject* exc = c.sstatus >= 400 ? status_error(c.sstatus, c.err_body)
                                       : conn_failed("stream closed: " + why, true, false);
      fail_stream_head(s, exc);
      Py_XDECREF(exc);
    }
    close_io(s);
    wake(s);
    return;
  }
  if (s->fut && c.state == kUntilClose) {  // a read-until-close body ends here
    std::string body;
    body.swap(c.body);
    c.close_after = true;
    finish_response(s, body.data(), body.size());
    close_io(s);
    return;
  }
  close_io(s);
  if (s->fut) {
    PyObject* f = s->fut;
    s->fut = nullptr;
    PyObject* exc = conn_failed("connection lost: " + why, !s->got_any, s->used > 1);
    pool_release(s);
    reject(f, exc);
    Py_XDECREF(exc);
    Py_DECREF(f);
  }
  pool_release(s);
}

// Write what is buffered.  false: the connection broke (already handled).
bool flush(ConnObject* s) {
  Core& c = *s->core;
  std::string err;
  while (c.wpos < c.wbuf.size()) {
    const long n = io_write(s, c.wbuf.data() + c.wpos, c.wbuf.size() - c.wpos, &err);
    if (n > 0) {
      c.wpos += static_cast<size_t>(n);
      continue;
    }
    if (n == kWantWrite) {
      set_writer(s, true);
      return true;
    }
    if (n == kWantRead) {  // TLS needs the peer first: the reader retries the write
      set_writer(s, false);
      return true;
    }
    lost(s, err);
    return false;
  }
  c.wbuf.clear();
  c.wpos = 0;
  set_writer(s, false);
  return true;
}

void handshake_step(ConnObject* s) {
  ERR_clear_error();
  errno = 0;
  const int r = SSL_connect(s->ssl);
  if (r == 1) {
    s->hs = kHsNone;
    set_writer(s, false);
    PyObject* f = s->hs_fut;
    s->hs_fut = nullptr;
    resolve(f, Py_None);
    Py_XDECREF(f);
    return;
  }
  const int e = SSL_get_error(s->ssl, r);
  if (e == SSL_ERROR_WANT_READ) {
    set_writer(s, false);
    return;
  }
  if (e == SSL_ERROR_WANT_WRITE) {
    set_writer(s, true);
    return;
  }
  const std::string msg = ssl_error_string(s->ssl, e);
  s->hs = kHsNone;
  close_io(s);
  PyObject* f = s->hs_fut;
  s->hs_fut = nullptr;
  PyObject* exc = ssl_error("TLS handshake failed: " + msg);
  reject(f, exc);
  Py_XDECREF(exc);
  Py_XDECREF(f);
}

void read_ready(ConnObject* s) {
  Core& c = *s->core;
  std::string err;
  size_t total = 0;
  bool eof = false, failed = false;
  for (;;) {
    const long n = io_read(s, g_rbuf, sizeof g_rbuf, &err);
    if (n > 0) {
      s->got_any = true;
      if (c.rpos == c.rbuf.size()) {
        c.rbuf.clear();
        c.rpos = 0;
      }
      c.rbuf.append(g_rbuf, static_cast<size_t>(n));
      total += static_cast<size_t>(n);
      // plain sockets: a short read drained the socket (the loop is level-triggered, so more
      // data wakes us again); TLS: read until OpenSSL needs the socket, it may hold records
      if (!s->ssl && static_cast<size_t>(n) < sizeof g_rbuf) break;
      // past the per-wake bound, stop only if the rest is still in the kernel (the loop wakes us
      // again); records OpenSSL already pulled off the socket would not wake anyone
      if (total >= kMaxReadPerWake && (!s->ssl || !SSL_has_pending(s->ssl))) break;
      continue;
    }
    if (n == 0) eof = true;
    else if (n == kWantWrite) set_writer(s, true);  // TLS renegotiation needs to write first
    else if (n == kIoError) failed = true;
    break;
  }
  if (total) {
    int r;
    if (s->mode == kStream) r = parse_stream(s);
    else {
      r = 1;
      while (r == 1 && s->fd >= 0) r = parse_response(s);  // stray bytes after a response stay buffered
      if (r == -1) {
        s->alive = false;
        close_io(s);
        if (s->fut) {
          PyObject* f = s->fut;
          s->fut = nullptr;
          PyObject* exc = conn_failed("bad HTTP response", false, false);
          pool_release(s);
          reject(f, exc);
          Py_XDECREF(exc);
          Py_DECREF(f);
        }
        return;
      }
    }
    if (r == -1) {  // stream ended by a decode error or bad head
      close_io(s);
      wake(s);
      return;
    }
  }
  if (s->fd < 0) return;
  if (eof) lost(s, "closed by peer");
  else if (failed) lost(s, err);
}

// ----------------------------------------------------------------------------- the type

// ----------------------------------------------------------------------------- TlsContext

// An SSL_CTX built here from PEM bytes, so the TLS state and the code driving it come from
// one libssl whatever OpenSSL the interpreter's own ssl module uses.
struct TlsCtxObject {
  PyObject_HEAD
  SSL_CTX* ctx;
};

PyTypeObject TlsCtxType = {
    PyVarObject_HEAD_INIT(nullptr, 0)
    "_netconn.TlsContext",                 /* tp_name */
    sizeof(TlsCtxObject),                  /* tp_basicsize */
};

std::string openssl_errors() {
  std::string msg;
  char buf[256];
  unsigned long e;
  while ((e = ERR_get_error()) != 0) {
    ERR_error_string_n(e, buf, sizeof buf);
    if (!msg.empty()) msg += "; ";
    msg += buf;
  }
  return msg;
}

int tls_fail(const std::string& what) {
  const std::string msg = what + (ERR_peek_error() ? ": " + openssl_errors() : std::string());
  if (g_ssl_error) {
    PyObject* exc = ssl_error(msg);
    if (exc) {
      PyErr_SetObject(reinterpret_cast<PyObject*>(Py_TYPE(exc)), exc);
      Py_DECREF(exc);
    }
  } else {
    PyErr_SetString(PyExc_ValueError, msg.c_str());
  }
  return -1;
}

// Every certificate of a PEM bundle into the context's trust store; -1 on none or a bad one.
int add_ca_pem(SSL_CTX* ctx, const char* data, Py_ssize_t len) {
  BIO* bio = BIO_new_mem_buf(data, static_cast<int>(len));
  if (!bio) return tls_fail("BIO_new_mem_buf failed");
  X509_STORE* store = SSL_CTX_get_cert_store(ctx);
  int n = 0;
  for (;;) {
    X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
    if (!x) break;
    const int ok = X509_STORE_add_cert(store, x);
    X509_free(x);
    if (ok != 1) {
      BIO_free(bio);
      return tls_fail("cannot add a CA certificate");
    }
    ++n;
  }
  BIO_free(bio);
  if (n == 0) return tls_fail("no CA certificate in the certificate-authority data");
  ERR_clear_error();  // the PEM end-of-data "error" after the last certificate
  return 0;
}

// The client certificate (first PEM block), its chain (the rest) and the private key.
int use_client_pem(SSL_CTX* ctx, const char* cert, Py_ssize_t cert_len, const char* key, Py_ssize_t key_len) {
  BIO* bio = BIO_new_mem_buf(cert, static_cast<int>(cert_len));
  if (!bio) return tls_fail("BIO_new_mem_buf failed");
  X509* leaf = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
  if (!leaf || SSL_CTX_use_certificate(ctx, leaf) != 1) {
    if (leaf) X509_free(leaf);
    BIO_free(bio);
    return tls_fail("cannot load the client certificate");
  }
  X509_free(leaf);
  for (;;) {
    X509* x = PEM_read_bio_X509(bio, nullptr, nullptr, nullptr);
    if (!x) break;
    if (SSL_CTX_add_extra_chain_cert(ctx, x) != 1) {  // takes ownership on success
      X509_free(x);
      BIO_free(bio);
      return tls_fail("cannot add a client chain certificate");
    }
  }
  BIO_free(bio);
  ERR_clear_error();
  // the key: its own data, or a PEM bundle holding certificate and key together
  bio = key_len > 0 ? BIO_new_mem_buf(key, static_cast<int>(key_len))
                    : BIO_new_mem_buf(cert, static_cast<int>(cert_len));
  if (!bio) return tls_fail("BIO_new_mem_buf failed");
  EVP_PKEY* pk = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  if (!pk || SSL_CTX_use_PrivateKey(ctx, pk) != 1) {
    if (pk) EVP_PKEY_free(pk);
    return tls_fail("cannot load the client key");
  }
  EVP_PKEY_free(pk);
  if (SSL_CTX_check_private_key(ctx) != 1) return tls_fail("the client key does not match its certificate");
  return 0;
}

// TlsContext(cadata=None, cafile=None, certdata=None, keydata=None, verify=True)
int tls_init(TlsCtxObject* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"cadata", "cafile", "certdata", "keydata", "verify", nullptr};
  const char *ca = nullptr, *cafile = nullptr, *cert = nullptr, *key = nullptr;
  Py_ssize_t ca_len = 0, cert_len = 0, key_len = 0;
  int verify = 1;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "|z#zz#z#p", const_cast<char**>(kwlist), &ca, &ca_len, &cafile,
                                   &cert, &cert_len, &key, &key_len, &verify))
    return -1;
  if (self->ctx) {
    PyErr_SetString(PyExc_RuntimeError, "TlsContext is already initialised");
    return -1;
  }
  SSL_CTX* ctx = SSL_CTX_new(TLS_client_method());
  if (!ctx) return tls_fail("SSL_CTX_new failed");
  self->ctx = ctx;  // freed by dealloc on any failure below
  SSL_CTX_set_min_proto_version(ctx, TLS1_2_VERSION);
  SSL_CTX_set_options(ctx, SSL_OP_NO_COMPRESSION);
  SSL_CTX_set_mode(ctx, SSL_MODE_RELEASE_BUFFERS);
  if (verify) {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_PEER, nullptr);
    if (ca && ca_len > 0) {
      if (add_ca_pem(ctx, ca, ca_len) < 0) return -1;
    } else if (cafile && *cafile) {
      if (SSL_CTX_load_verify_locations(ctx, cafile, nullptr) != 1) return tls_fail("cannot load the CA file");
    } else if (SSL_CTX_set_default_verify_paths(ctx) != 1) {
      return tls_fail("cannot load the system CA certificates");
    }
  } else {
    SSL_CTX_set_verify(ctx, SSL_VERIFY_NONE, nullptr);
  }
  if (cert && cert_len > 0 && use_client_pem(ctx, cert, cert_len, key, key_len) < 0) return -1;
  static const unsigned char kAlpn[] = {8, 'h', 't', 't', 'p', '/', '1', '.', '1'};
  if (SSL_CTX_set_alpn_protos(ctx, kAlpn, sizeof kAlpn) != 0) return tls_fail("cannot set ALPN");
  return 0;
}

void tls_dealloc(TlsCtxObject* self) {
  if (self->ctx) SSL_CTX_free(self->ctx);
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

PyObject* tls_verify(TlsCtxObject* self, void*) {
  if (!self->ctx) Py_RETURN_NONE;
  return PyBool_FromLong((SSL_CTX_get_verify_mode(self->ctx) & SSL_VERIFY_PEER) != 0);
}

PyGetSetDef kTlsGetSet[] = {
    {"verify", reinterpret_cast<getter>(tls_verify), nullptr, "peer certificates are verified", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr},
};

SSL_CTX* ssl_ctx_of(PyObject* ctx) {
  // A TlsContext built here, or -- only when configure() proved CPython's _ssl shares this
  // extension's libssl -- the SSL_CTX of an ssl.SSLContext: _ssl._SSLContext's C struct starts
  // with the SSL_CTX pointer right after the object header, and the match with the
  // Python-visible options and verify mode guards that layout assumption.
  if (PyObject_TypeCheck(ctx, &TlsCtxType)) {
    SSL_CTX* sc = reinterpret_cast<TlsCtxObject*>(ctx)->ctx;
    if (!sc) PyErr_SetString(PyExc_ValueError, "TlsContext is not initialised");
    return sc;
  }
  bool is_ctx = false;
  for (PyTypeObject* t = Py_TYPE(ctx); t; t = t->tp_base)
    if (std::strcmp(t->tp_name, "_ssl._SSLContext") == 0) {
      is_ctx = true;
      break;
    }
  if (!is_ctx) {
    PyErr_SetString(PyExc_TypeError, "ssl_context must be a TlsContext or an ssl.SSLContext");
    return nullptr;
  }
  if (!g_shared_openssl) {
    PyErr_SetString(PyExc_TypeError, "CPython's ssl module uses another OpenSSL than _netconn");
    return nullptr;
  }
  SSL_CTX* sc = *reinterpret_cast<SSL_CTX**>(reinterpret_cast<char*>(ctx) + sizeof(PyObject));
  if (!sc) {
    PyErr_SetString(PyExc_TypeError, "SSLContext has no SSL_CTX");
    return nullptr;
  }
  PyObject* opt = PyObject_GetAttr(ctx, s_options);
  PyObject* vm = opt ? PyObject_GetAttr(ctx, s_verify_mode) : nullptr;
  if (!vm) {
    Py_XDECREF(opt);
    return nullptr;
  }
  const unsigned long long py_opt = PyLong_AsUnsignedLongLong(opt);
  const long py_vm = PyLong_AsLong(vm);
  Py_DECREF(opt);
  Py_DECREF(vm);
  if (PyErr_Occurred()) return nullptr;
  const int mode = SSL_CTX_get_verify_mode(sc);
  const int want = py_vm == 0 ? SSL_VERIFY_NONE
                   : py_vm == 1 ? SSL_VERIFY_PEER
                                : (SSL_VERIFY_PEER | SSL_VERIFY_FAIL_IF_NO_PEER_CERT);
  if (static_cast<unsigned long long>(SSL_CTX_get_options(sc)) != py_opt || mode != want) {
    PyErr_SetString(PyExc_TypeError, "unrecognised SSLContext layout");
    return nullptr;
  }
  return sc;
}

int conn_init(ConnObject* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"loop", "fd", "ssl_context", "server_hostname", "check_hostname",
                                 "hostname_checks_common_name", nullptr};
  PyObject *loop, *ctx = Py_None;
  int fd, check_hostname = 0, checks_cn = 1;
  const char* host = nullptr;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "Oi|Ozpp", const_cast<char**>(kwlist), &loop, &fd, &ctx, &host,
                                   &check_hostname, &checks_cn))
    return -1;
  if (self->core) {
    PyErr_SetString(PyExc_RuntimeError, "Conn is already initialised");
    return -1;
  }
  if (!g_conn_failed) {
    PyErr_SetString(PyExc_RuntimeError, "_netconn.configure() was not called");
    return -1;
  }
  SSL* ssl = nullptr;
  if (ctx != Py_None) {
    SSL_CTX* sc = ssl_ctx_of(ctx);
    if (!sc) return -1;
    ssl = SSL_new(sc);
    if (!ssl || SSL_set_fd(ssl, fd) != 1) {
      if (ssl) SSL_free(ssl);
      PyErr_SetString(PyExc_RuntimeError, "SSL_new failed");
      return -1;
    }
    SSL_set_connect_state(ssl);
    SSL_set_mode(ssl, SSL_MODE_ENABLE_PARTIAL_WRITE | SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    SSL_set_options(ssl, SSL_OP_IGNORE_UNEXPECTED_EOF);
    if (host && *host) {
      unsigned char tmp[16];
      const bool ip = inet_pton(AF_INET, host, tmp) == 1 || inet_pton(AF_INET6, host, tmp) == 1;
      if (!ip) SSL_set_tlsext_host_name(ssl, host);  // SNI is for names only (RFC 6066)
      if (check_hostname) {
        X509_VERIFY_PARAM* p = SSL_get0_param(ssl);
        X509_VERIFY_PARAM_set_hostflags(
            p, X509_CHECK_FLAG_NO_PARTIAL_WILDCARDS | (checks_cn ? 0 : X509_CHECK_FLAG_NEVER_CHECK_SUBJECT));
        const int ok = ip ? X509_VERIFY_PARAM_set1_ip_asc(p, host) : X509_VERIFY_PARAM_set1_host(p, host, 0);
        if (ok != 1) {
          SSL_free(ssl);
          PyErr_Format(PyExc_ValueError, "invalid server hostname %s", host);
          return -1;
        }
      }
    } else if (check_hostname) {
      SSL_free(ssl);
      PyErr_SetString(PyExc_ValueError, "check_hostname requires server_hostname");
      return -1;
    }
  }
  self->core = new Core();
  Py_INCREF(loop);
  self->loop = loop;
  if (ssl) {
    Py_INCREF(ctx);
    self->ssl_ctx = ctx;
  }
  self->ssl = ssl;
  self->fd = fd;
  self->alive = true;
  set_reader(self, true);
  if (!self->reader_on) {
    PyErr_SetString(PyExc_RuntimeError, "loop.add_reader failed");
    close_io(self);
    return -1;
  }
  return 0;
}

PyObject* conn_new(PyTypeObject* type, PyObject*, PyObject*) {
  ConnObject* self = reinterpret_cast<ConnObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->fd = -1;
  return reinterpret_cast<PyObject*>(self);
}

int conn_traverse(ConnObject* self, visitproc visit, void* arg) {
  Py_VISIT(self->loop);
  Py_VISIT(self->ssl_ctx);
  Py_VISIT(self->hs_fut);
  Py_VISIT(self->fut);
  Py_VISIT(self->decode);
  Py_VISIT(self->items);
  Py_VISIT(self->waiter);
  Py_VISIT(self->stream_error);
  Py_VISIT(self->pool);
  return 0;
}

int conn_clear(ConnObject* self) {
  Py_CLEAR(self->hs_fut);
  Py_CLEAR(self->fut);
  Py_CLEAR(self->decode);
  Py_CLEAR(self->items);
  Py_CLEAR(self->waiter);
  Py_CLEAR(self->stream_error);
  Py_CLEAR(self->ssl_ctx);
  Py_CLEAR(self->loop);
  Py_CLEAR(self->pool);
  return 0;
}

void conn_dealloc(ConnObject* self) {
  PyObject_GC_UnTrack(self);
  if (self->weakrefs) PyObject_ClearWeakRefs(reinterpret_cast<PyObject*>(self));
  // the loop no longer holds our callbacks (they hold a reference to us): just release
  if (self->ssl) SSL_free(self->ssl);
  if (self->fd >= 0) ::close(self->fd);
  conn_clear(self);
  delete self->core;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

bool check_ready(ConnObject* self) {
  if (!self->core) {
    PyErr_SetString(PyExc_RuntimeError, "Conn is not initialised");
    return false;
  }
  return true;
}

PyObject* new_future(ConnObject* self) {
  if (!self->loop) {
    PyErr_SetString(PyExc_RuntimeError, "Conn has no event loop");
    return nullptr;
  }
  return PyObject_CallMethodNoArgs(self->loop, s_create_future);
}

PyObject* failed_future(ConnObject* self, PyObject* exc) {
  PyObject* f = new_future(self);
  if (f && exc) {
    PyObject* r = PyObject_CallMethodOneArg(f, s_set_exception, exc);
    Py_XDECREF(r);
    if (!r) Py_CLEAR(f);
  }
  Py_XDECREF(exc);
  return f;
}

// handshake() -> Future[None]: the TLS handshake (a plain connection returns a done future)
PyObject* conn_handshake(ConnObject* self, PyObject*) {
  if (!check_ready(self)) return nullptr;
  if (!self->ssl) {
    PyObject* f = new_future(self);
    if (f) resolve(f, Py_None);
    return f;
  }
  if (self->fd < 0) return failed_future(self, ssl_error("TLS handshake on a closed connection"));
  if (self->hs_fut) {
    Py_INCREF(self->hs_fut);
    return self->hs_fut;
  }
  PyObject* f = new_future(self);
  if (!f) return nullptr;
  Py_INCREF(f);
  self->hs_fut = f;
  self->hs = kHsRunning;
  Py_INCREF(self);
  handshake_step(self);
  Py_DECREF(self);
  return f;
}

// Queue ``data`` and write what the socket takes now.
bool start_write(ConnObject* self, PyObject* data) {
  Py_buffer view;
  if (PyObject_GetBuffer(data, &view, PyBUF_SIMPLE) < 0) return false;
  Core& c = *self->core;
  c.wbuf.append(static_cast<const char*>(view.buf), static_cast<size_t>(view.len));
  PyBuffer_Release(&view);
  if (!self->writer_on) flush(self);
  return true;
}

// send(data) -> Future[(status, body, retry_after)]
PyObject* conn_send(ConnObject* self, PyObject* data) {
  if (!check_ready(self)) return nullptr;
  if (self->mode != kRequest) {
    PyErr_SetString(PyExc_RuntimeError, "send() on a stream connection");
    return nullptr;
  }
  if (self->fd < 0 || !self->alive)
    return failed_future(self, conn_failed("connection is closed", true, self->used > 0));
  if (self->fut) {
    PyErr_SetString(PyExc_RuntimeError, "a request is already in flight on this connection");
    return nullptr;
  }
  PyObject* f = new_future(self);
  if (!f) return nullptr;
  Py_INCREF(f);
  self->fut = f;
  self->used += 1;
  self->got_any = false;
  Py_INCREF(self);
  const bool ok = start_write(self, data);
  Py_DECREF(self);
  if (!ok) {
    Py_CLEAR(self->fut);
    Py_DECREF(f);
    return nullptr;
  }
  return f;
}

// open_stream(data, decode) -> Future[int status]
PyObject* conn_open_stream(ConnObject* self, PyObject* args) {
  PyObject *data, *decode;
  if (!PyArg_ParseTuple(args, "OO", &data, &decode)) return nullptr;
  if (!check_ready(self)) return nullptr;
  if (self->mode != kRequest || self->used) {
    PyErr_SetString(PyExc_RuntimeError, "open_stream() needs a fresh connection");
    return nullptr;
  }
  if (self->fd < 0 || !self->alive)
    return failed_future(self, conn_failed("stream closed: connection is closed", true, false));
  PyObject* items = PyList_New(0);
  PyObject* f = items ? new_future(self) : nullptr;
  if (!f) {
    Py_XDECREF(items);
    return nullptr;
  }
  self->mode = kStream;
  self->items = items;
  Py_INCREF(decode);
  self->decode = decode;
  Py_INCREF(f);
  self->fut = f;
  self->used = 1;
  Py_INCREF(self);
  const bool ok = start_write(self, data);
  Py_DECREF(self);
  if (!ok) {
    Py_CLEAR(self->fut);
    Py_DECREF(f);
    return nullptr;
  }
  return f;
}

PyObject* conn_on_readable(ConnObject* self, PyObject*) {
  if (!self->core || self->fd < 0) Py_RETURN_NONE;
  Py_INCREF(self);  // completing futures may drop the last outside reference
  if (self->hs == kHsRunning) handshake_step(self);
  else {
    if (self->core->wpos < self->core->wbuf.size() && !self->writer_on) flush(self);
    if (self->fd >= 0) read_ready(self);
  }
  Py_DECREF(self);
  Py_RETURN_NONE;
}

PyObject* conn_on_writable(ConnObject* self, PyObject*) {
  if (!self->core || self->fd < 0) Py_RETURN_NONE;
  Py_INCREF(self);
  if (self->hs == kHsRunning) handshake_step(self);
  else flush(self);
  Py_DECREF(self);
  Py_RETURN_NONE;
}

// close(): unregister and close the socket; a pending response or stream head fails like a
// connection the peer closed
PyObject* conn_close(ConnObject* self, PyObject*) {
  if (!self->core) Py_RETURN_NONE;
  Py_INCREF(self);
  if (self->fd >= 0) lost(self, "closed");
  else {
    self->alive = false;
    if (self->mode == kStream) {
      self->stream_done = true;
      wake(self);
    }
  }
  if (self->hs_fut) {
    PyObject* f = self->hs_fut;
    self->hs_fut = nullptr;
    PyObject* exc = ssl_error("connection closed during the TLS handshake");
    reject(f, exc);
    Py_XDECREF(exc);
    Py_DECREF(f);
  }
  pool_release(self);
  Py_DECREF(self);
  Py_RETURN_NONE;
}

PyObject* conn_closing(ConnObject* self, PyObject*) { return PyBool_FromLong(self->fd < 0 || !self->alive); }

// take() -> list: every decoded item not taken yet
PyObject* conn_take(ConnObject* self, PyObject*) {
  if (!self->items || PyList_GET_SIZE(self->items) == 0) return PyList_New(0);
  PyObject* fresh = PyList_New(0);
  if (!fresh) return nullptr;
  PyObject* out = self->items;
  self->items = fresh;
  return out;
}

// take_one() -> item | None
PyObject* conn_take_one(ConnObject* self, PyObject*) {
  if (!self->items || PyList_GET_SIZE(self->items) == 0) Py_RETURN_NONE;
  PyObject* item = PyList_GET_ITEM(self->items, 0);
  Py_INCREF(item);
  if (PySequence_DelItem(self->items, 0) < 0) {
    Py_DECREF(item);
    return nullptr;
  }
  return item;
}

// wait() -> Future | None: None when items are ready or the stream has ended
PyObject* conn_wait(ConnObject* self, PyObject*) {
  if (!check_ready(self)) return nullptr;
  if ((self->items && PyList_GET_SIZE(self->items) > 0) || self->stream_done || self->fd < 0) Py_RETURN_NONE;
  if (self->waiter) {  // a waiter cancelled with its awaiting task is replaced
    PyObject* d = PyObject_CallMethodNoArgs(self->waiter, s_done);
    if (!d) return nullptr;
    const bool done = d == Py_True;
    Py_DECREF(d);
    if (done) Py_CLEAR(self->waiter);
  }
  if (!self->waiter) {
    self->waiter = new_future(self);
    if (!self->waiter) return nullptr;
  }
  Py_INCREF(self->waiter);
  return self->waiter;
}

PyObject* get_alive(ConnObject* self, void*) { return PyBool_FromLong(self->alive && self->fd >= 0); }

int set_alive(ConnObject* self, PyObject* v, void*) {
  if (!v) {
    PyErr_SetString(PyExc_AttributeError, "cannot delete alive");
    return -1;
  }
  const int t = PyObject_IsTrue(v);
  if (t < 0) return -1;
  self->alive = t && self->fd >= 0;
  return 0;
}

PyObject* get_fut(ConnObject* self, void*) {
  PyObject* f = self->fut ? self->fut : Py_None;
  Py_INCREF(f);
  return f;
}

PyObject* get_done(ConnObject* self, void*) { return PyBool_FromLong(self->stream_done || self->fd < 0); }

PyObject* get_error(ConnObject* self, void*) {
  PyObject* e = self->stream_error ? self->stream_error : Py_None;
  Py_INCREF(e);
  return e;
}

PyObject* get_pending(ConnObject* self, void*) {
  return PyLong_FromSsize_t(self->items ? PyList_GET_SIZE(self->items) : 0);
}

PyObject* get_tls(ConnObject* self, void*) { return PyBool_FromLong(self->ssl != nullptr); }

PyObject* get_tls_version(ConnObject* self, void*) {
  if (!self->ssl) Py_RETURN_NONE;
  return PyUnicode_FromString(SSL_get_version(self->ssl));
}

PyObject* get_alpn(ConnObject* self, void*) {
  if (!self->ssl) Py_RETURN_NONE;
  const unsigned char* p = nullptr;
  unsigned int n = 0;
  SSL_get0_alpn_selected(self->ssl, &p, &n);
  if (!p || !n) Py_RETURN_NONE;
  return PyUnicode_FromStringAndSize(reinterpret_cast<const char*>(p), n);
}

PyMethodDef kConnMethods[] = {
    {"handshake", reinterpret_cast<PyCFunction>(conn_handshake), METH_NOARGS,
     "handshake() -> Future[None]: run the TLS handshake (plain connections: a done future)"},
    {"send", reinterpret_cast<PyCFunction>(conn_send), METH_O,
     "send(data) -> Future[(status, body, retry_after)]: one request/response exchange"},
    {"open_stream", reinterpret_cast<PyCFunction>(conn_open_stream), METH_VARARGS,
     "open_stream(data, decode) -> Future[status]: turn the connection into a line stream"},
    {"take", reinterpret_cast<PyCFunction>(conn_take), METH_NOARGS, "take() -> list of decoded items"},
    {"take_one", reinterpret_cast<PyCFunction>(conn_take_one), METH_NOARGS, "take_one() -> item or None"},
    {"wait", reinterpret_cast<PyCFunction>(conn_wait), METH_NOARGS,
     "wait() -> Future or None (None: items ready or the stream ended)"},
    {"close", reinterpret_cast<PyCFunction>(conn_close), METH_NOARGS, "close the connection"},
    {"closing", reinterpret_cast<PyCFunction>(conn_closing), METH_NOARGS, "closed or marked dead"},
    {"_on_readable", reinterpret_cast<PyCFunction>(conn_on_readable), METH_NOARGS, "loop reader callback"},
    {"_on_writable", reinterpret_cast<PyCFunction>(conn_on_writable), METH_NOARGS, "loop writer callback"},
    {nullptr, nullptr, 0, nullptr},
};

PyGetSetDef kConnGetSet[] = {
    {"alive", reinterpret_cast<getter>(get_alive), reinterpret_cast<setter>(set_alive),
     "usable for another request", nullptr},
    {"fut", reinterpret_cast<getter>(get_fut), nullptr, "the in-flight response future, or None", nullptr},
    {"done", reinterpret_cast<getter>(get_done), nullptr, "stream mode: the stream has ended", nullptr},
    {"error", reinterpret_cast<getter>(get_error), nullptr, "stream mode: what ended the stream", nullptr},
    {"pending", reinterpret_cast<getter>(get_pending), nullptr, "stream mode: items not taken yet", nullptr},
    {"tls", reinterpret_cast<getter>(get_tls), nullptr, "TLS connection", nullptr},
    {"tls_version", reinterpret_cast<getter>(get_tls_version), nullptr, "negotiated TLS version", nullptr},
    {"alpn", reinterpret_cast<getter>(get_alpn), nullptr, "negotiated ALPN protocol", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr},
};

PyMemberDef kConnMembers[] = {
    {"used", T_LONG, offsetof(ConnObject, used), READONLY, "requests sent"},
    {"fd", T_INT, offsetof(ConnObject, fd), READONLY, "socket file descriptor (-1 once closed)"},
    {"ssl_gen", T_LONG, offsetof(ConnObject, ssl_gen), 0, "pool bookkeeping: TLS context generation"},
    {"deadline", T_DOUBLE, offsetof(ConnObject, deadline), 0, "pool bookkeeping: response due (loop time)"},
    {nullptr, 0, 0, 0, nullptr},
};

PyTypeObject ConnType = {
    PyVarObject_HEAD_INIT(nullptr, 0)
    "_netconn.Conn",                       /* tp_name */
    sizeof(ConnObject),                    /* tp_basicsize */
};

// ----------------------------------------------------------------------------- the pool

double monotonic_now() {  // asyncio's loop.time() is time.monotonic(): CLOCK_MONOTONIC
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<double>(ts.tv_sec) + static_cast<double>(ts.tv_nsec) * 1e-9;
}

void pool_release(ConnObject* s) {
  PoolObject* p = reinterpret_cast<PoolObject*>(s->pool);
  if (!p) return;
  s->pool = nullptr;  // our reference to p, released at the end
  std::vector<ConnObject*>& busy = *p->busy;
  bool owned = false;  // the busy list's reference to s
  for (size_t i = 0; i < busy.size(); ++i)
    if (busy[i] == s) {
      busy[i] = busy.back();
      busy.pop_back();
      owned = true;
      break;
    }
  if (owned) {
    if (s->alive && s->fd >= 0 && !s->fut && !p->closed && s->ssl_gen == p->ssl_gen &&
        static_cast<Py_ssize_t>(p->idle->size()) < p->max_idle) {
      p->idle->push_back(s);  // the reference moves to the idle list
    } else {
      close_io(s);
      Py_DECREF(s);
    }
  }
  Py_DECREF(p);
}

// The latin-1 bytes of str `o` appended to `out` (the encoding of the Python request head).
bool append_latin1(std::string* out, PyObject* o) {
  if (!PyUnicode_Check(o)) {
    PyErr_SetString(PyExc_TypeError, "expected str");
    return false;
  }
  if (PyUnicode_IS_COMPACT_ASCII(o)) {
    out->append(reinterpret_cast<const char*>(PyUnicode_DATA(o)), static_cast<size_t>(PyUnicode_GET_LENGTH(o)));
    return true;
  }
  PyObject* b = PyUnicode_AsLatin1String(o);
  if (!b) return false;
  out->append(PyBytes_AS_STRING(b), static_cast<size_t>(PyBytes_GET_SIZE(b)));
  Py_DECREF(b);
  return true;
}

// The request: "<method> <target><path> HTTP/1.1", the fixed headers, Accept, and the body
// with its Content-Type and Content-Length (POST/PUT/PATCH without a body send length 0).
bool build_request(PoolObject* p, PyObject* const* a, std::string* out) {
  PyObject *method = a[0], *path = a[1], *body = a[2], *ctype = a[3], *accept = a[4];
  Py_buffer view;
  const bool has_body = body != Py_None;
  if (has_body && PyObject_GetBuffer(body, &view, PyBUF_SIMPLE) < 0) return false;
  out->reserve(256 + p->fixed->size() + (has_body ? static_cast<size_t>(view.len) : 0));
  bool ok = append_latin1(out, method);
  if (ok) {
    out->push_back(' ');
    out->append(*p->target);
    ok = append_latin1(out, path);
  }
  if (ok) {
    out->append(" HTTP/1.1\r\n");
    out->append(*p->fixed);
    out->append("Accept: ");
    ok = append_latin1(out, accept);
  }
  if (ok) {
    out->append("\r\n");
    if (has_body) {
      out->append("Content-Type: ");
      ok = append_latin1(out, ctype);
      if (ok) {
        out->append("\r\nContent-Length: ");
        out->append(std::to_string(view.len));
        out->append("\r\n\r\n");
        out->append(static_cast<const char*>(view.buf), static_cast<size_t>(view.len));
      }
    } else {
      const char* m = PyUnicode_Check(method) ? PyUnicode_AsUTF8(method) : nullptr;
      if (!m) ok = false;
      else if (!std::strcmp(m, "POST") || !std::strcmp(m, "PUT") || !std::strcmp(m, "PATCH"))
        out->append("Content-Length: 0\r\n\r\n");
      else out->append("\r\n");
    }
  }
  if (has_body) PyBuffer_Release(&view);
  return ok;
}

// Send `req` on `c` (request mode, nothing in flight) as a request of pool `p`: `c` joins the
// busy list (taking over the caller's reference) until its response completes.
PyObject* pool_start(PoolObject* p, ConnObject* c, const std::string& req) {
  PyObject* f = new_future(c);
  if (!f) {
    PyObject *type, *value, *tb;
    PyErr_Fetch(&type, &value, &tb);
    close_io(c);  // neither pooled nor in flight any more: unregister it
    PyErr_Restore(type, value, tb);
    Py_DECREF(c);
    return nullptr;
  }
  Py_INCREF(f);
  c->fut = f;
  c->used += 1;
  c->got_any = false;
  c->deadline = monotonic_now() + p->timeout;
  Py_INCREF(p);
  c->pool = reinterpret_cast<PyObject*>(p);
  p->busy->push_back(c);  // the caller's reference
  Py_INCREF(c);           // ours, while we write (a failed write releases it from the pool)
  c->core->wbuf.append(req);
  if (!c->writer_on) flush(c);
  Py_DECREF(c);
  return f;
}

PyObject* pool_new(PyTypeObject* type, PyObject*, PyObject*) {
  PoolObject* self = reinterpret_cast<PoolObject*>(type->tp_alloc(type, 0));
  if (!self) return nullptr;
  self->idle = new std::vector<ConnObject*>();
  self->busy = new std::vector<ConnObject*>();
  self->target = new std::string();
  self->fixed = new std::string();
  self->max_idle = 64;
  self->timeout = 60.0;
  return reinterpret_cast<PyObject*>(self);
}

// Pool(max_idle, timeout)
int pool_init(PoolObject* self, PyObject* args, PyObject* kw) {
  static const char* kwlist[] = {"max_idle", "timeout", nullptr};
  Py_ssize_t max_idle = 64;
  double timeout = 60.0;
  if (!PyArg_ParseTupleAndKeywords(args, kw, "|nd", const_cast<char**>(kwlist), &max_idle, &timeout)) return -1;
  self->max_idle = max_idle;
  self->timeout = timeout;
  return 0;
}

// Drop every connection the pool holds (idle ones are closed; busy ones are closed too, their
// requests failing like a lost connection).
void pool_drop_all(PoolObject* self, bool busy_too) {
  std::vector<ConnObject*> idle;
  idle.swap(*self->idle);
  for (ConnObject* c : idle) {
    close_io(c);
    Py_DECREF(c);
  }
  if (!busy_too) return;
  while (!self->busy->empty()) {
    ConnObject* c = self->busy->back();
    Py_INCREF(c);
    if (c->pool) lost(c, "pool closed");  // releases c from the busy list
    else {
      self->busy->pop_back();  // cannot happen (busy entries point back here): keep the list finite
      Py_DECREF(c);
    }
    Py_DECREF(c);
  }
}

int pool_traverse(PoolObject* self, visitproc visit, void* arg) {
  if (self->idle)
    for (ConnObject* c : *self->idle) Py_VISIT(c);
  if (self->busy)
    for (ConnObject* c : *self->busy) Py_VISIT(c);
  return 0;
}

int pool_clear(PoolObject* self) {
  if (self->idle) {
    std::vector<ConnObject*> v;
    v.swap(*self->idle);
    for (ConnObject* c : v) Py_DECREF(c);
  }
  if (self->busy) {
    std::vector<ConnObject*> v;
    v.swap(*self->busy);
    for (ConnObject* c : v) Py_DECREF(c);
  }
  return 0;
}

void pool_dealloc(PoolObject* self) {
  PyObject_GC_UnTrack(self);
  if (self->weakrefs) PyObject_ClearWeakRefs(reinterpret_cast<PyObject*>(self));
  pool_clear(self);
  delete self->idle;
  delete self->busy;
  delete self->target;
  delete self->fixed;
  Py_TYPE(self)->tp_free(reinterpret_cast<PyObject*>(self));
}

// request(method, path, body, content_type, accept) -> Future[(status, body, retry_after)] | None
// (None: no idle connection -- the caller connects one and uses request_on)
PyObject* pool_request(PoolObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 5) {
    PyErr_SetString(PyExc_TypeError, "request(method, path, body, content_type, accept)");
    return nullptr;
  }
  ConnObject* c = nullptr;
  while (!self->idle->empty()) {
    ConnObject* t = self->idle->back();
    self->idle->pop_back();
    if (t->alive && t->fd >= 0 && !t->fut && t->core) {
      c = t;
      break;
    }
    close_io(t);
    Py_DECREF(t);
  }
  if (!c) Py_RETURN_NONE;
  std::string req;
  if (!build_request(self, args, &req)) {
    self->idle->push_back(c);  // unused: back where it was
    return nullptr;
  }
  return pool_start(self, c, req);
}

// request_on(conn, method, path, body, content_type, accept) -> Future: the same on a fresh connection
PyObject* pool_request_on(PoolObject* self, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 6 || !PyObject_TypeCheck(args[0], &ConnType)) {
    PyErr_SetString(PyExc_TypeError, "request_on(conn, method, path, body, content_type, accept)");
    return nullptr;
  }
  ConnObject* c = reinterpret_cast<ConnObject*>(args[0]);
  if (!check_ready(c)) return nullptr;
  if (c->mode != kRequest || c->fut || c->pool) {
    PyErr_SetString(PyExc_RuntimeError, "request_on() needs an idle request connection");
    return nullptr;
  }
  std::string req;
  if (!build_request(self, args + 1, &req)) {
    // a fresh connection nobody else holds: do not leave it registered with the loop
    PyObject *type, *value, *tb;
    PyErr_Fetch(&type, &value, &tb);  // closing calls into the loop: keep the error aside
    close_io(c);
    PyErr_Restore(type, value, tb);
    return nullptr;
  }
  if (c->fd < 0 || !c->alive) return failed_future(c, conn_failed("connection is closed", true, c->used > 0));
  Py_INCREF(c);
  return pool_start(self, c, req);
}

// sweep(now) -> int: fail the requests whose deadline passed (asyncio.TimeoutError, connection
// closed); returns how many are still in flight
PyObject* pool_sweep(PoolObject* self, PyObject* arg) {
  const double now = PyFloat_AsDouble(arg);
  if (now == -1.0 && PyErr_Occurred()) return nullptr;
  std::vector<ConnObject*> late;
  for (ConnObject* c : *self->busy)
    if (c->deadline <= now) {
      Py_INCREF(c);
      late.push_back(c);
    }
  for (ConnObject* c : late) {
    PyObject* f = c->fut;
    c->fut = nullptr;
    close_io(c);
    pool_release(c);
    if (f) {
      PyObject* exc = g_timeout_error ? PyObject_CallNoArgs(g_timeout_error) : nullptr;
      reject(f, exc);
      Py_XDECREF(exc);
      Py_DECREF(f);
    }
    Py_DECREF(c);
  }
  return PyLong_FromSsize_t(static_cast<Py_ssize_t>(self->busy->size()));
}

// discard(fut): the request of `fut` was abandoned (its caller was cancelled): close its connection
PyObject* pool_discard(PoolObject* self, PyObject* fut) {
  for (ConnObject* c : *self->busy)
    if (c->fut == fut) {
      Py_INCREF(c);
      lost(c, "request abandoned");
      Py_DECREF(c);
      break;
    }
  Py_RETURN_NONE;
}

// set_fixed(target, fixed): the request-target prefix and the header lines of every request
PyObject* pool_set_fixed(PoolObject* self, PyObject* args) {
  PyObject *target, *fixed;
  if (!PyArg_ParseTuple(args, "UU", &target, &fixed)) return nullptr;
  std::string t, f;
  if (!append_latin1(&t, target) || !append_latin1(&f, fixed)) return nullptr;
  self->target->swap(t);
  self->fixed->swap(f);
  Py_RETURN_NONE;
}

// close_idle(): close the idle connections (a rotated TLS context; busy ones close when done)
PyObject* pool_close_idle(PoolObject* self, PyObject*) {
  pool_drop_all(self, false);
  Py_RETURN_NONE;
}

// close(): no more reuse; idle connections close now, busy ones when their response completes
PyObject* pool_close(PoolObject* self, PyObject*) {
  self->closed = true;
  pool_drop_all(self, false);
  Py_RETURN_NONE;
}

// abort(): close every connection, failing the requests in flight
PyObject* pool_abort(PoolObject* self, PyObject*) {
  self->closed = true;
  pool_drop_all(self, true);
  Py_RETURN_NONE;
}

PyObject* pool_idle(PoolObject* self, PyObject*) {
  PyObject* out = PyList_New(static_cast<Py_ssize_t>(self->idle->size()));
  if (!out) return nullptr;
  for (size_t i = 0; i < self->idle->size(); ++i) {
    PyObject* c = reinterpret_cast<PyObject*>((*self->idle)[i]);
    Py_INCREF(c);
    PyList_SET_ITEM(out, static_cast<Py_ssize_t>(i), c);
  }
  return out;
}

PyObject* pool_get_busy(PoolObject* self, void*) { return PyLong_FromSize_t(self->busy->size()); }
PyObject* pool_get_closed(PoolObject* self, void*) { return PyBool_FromLong(self->closed); }

PyMethodDef kPoolMethods[] = {
    {"request", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(pool_request)), METH_FASTCALL,
     "request(method, path, body, content_type, accept) -> Future | None (no idle connection)"},
    {"request_on", reinterpret_cast<PyCFunction>(reinterpret_cast<void (*)(void)>(pool_request_on)), METH_FASTCALL,
     "request_on(conn, method, path, body, content_type, accept) -> Future"},
    {"sweep", reinterpret_cast<PyCFunction>(pool_sweep), METH_O, "sweep(now) -> requests still in flight"},
    {"discard", reinterpret_cast<PyCFunction>(pool_discard), METH_O, "discard(fut): close its connection"},
    {"set_fixed", reinterpret_cast<PyCFunction>(pool_set_fixed), METH_VARARGS, "set_fixed(target, fixed)"},
    {"close_idle", reinterpret_cast<PyCFunction>(pool_close_idle), METH_NOARGS, "close the idle connections"},
    {"close", reinterpret_cast<PyCFunction>(pool_close), METH_NOARGS, "stop reusing connections"},
    {"abort", reinterpret_cast<PyCFunction>(pool_abort), METH_NOARGS, "close everything, failing requests"},
    {"idle", reinterpret_cast<PyCFunction>(pool_idle), METH_NOARGS, "idle() -> list of idle connections"},
    {nullptr, nullptr, 0, nullptr},
};

PyGetSetDef kPoolGetSet[] = {
    {"busy", reinterpret_cast<getter>(pool_get_busy), nullptr, "requests in flight", nullptr},
    {"closed", reinterpret_cast<getter>(pool_get_closed), nullptr, "close() was called", nullptr},
    {nullptr, nullptr, nullptr, nullptr, nullptr},
};

PyMemberDef kPoolMembers[] = {
    {"ssl_gen", T_LONG, offsetof(PoolObject, ssl_gen), 0, "TLS context generation of reusable connections"},
    {"max_idle", T_PYSSIZET, offsetof(PoolObject, max_idle), 0, "idle connections kept"},
    {"timeout", T_DOUBLE, offsetof(PoolObject, timeout), 0, "seconds a response may take"},
    {nullptr, 0, 0, 0, nullptr},
};

PyTypeObject PoolType = {
    PyVarObject_HEAD_INIT(nullptr, 0)
    "_netconn.Pool",                       /* tp_name */
    sizeof(PoolObject),                    /* tp_basicsize */
};

// configure(ConnectionFailed, HttpStatusError, SSLError)
// Does CPython's _ssl extension (its file: `ssl_path`) resolve SSL_CTX_new to the very function
// this extension calls, and report the same OpenSSL build number?  Only then may an
// ssl.SSLContext's SSL_CTX be driven from here.
bool same_openssl(const char* ssl_path, unsigned long long py_version) {
  if (!ssl_path || !*ssl_path) return false;
  if (py_version != static_cast<unsigned long long>(OpenSSL_version_num())) return false;
  void* h = dlopen(ssl_path, RTLD_NOW | RTLD_NOLOAD);
  if (!h) return false;
  void* theirs = dlsym(h, "SSL_CTX_new");
  dlclose(h);
  return theirs != nullptr && theirs == reinterpret_cast<void*>(&SSL_CTX_new);
}

// configure(ConnectionFailed, HttpStatusError, SSLError[, TimeoutError[, ssl_module_path,
//           ssl_openssl_version_number]])
PyObject* configure(PyObject*, PyObject* args) {
  PyObject *cf, *se, *sslerr, *te = nullptr;
  const char* ssl_path = nullptr;
  unsigned long long py_version = 0;
  if (!PyArg_ParseTuple(args, "OOO|OzK", &cf, &se, &sslerr, &te, &ssl_path, &py_version)) return nullptr;
  Py_INCREF(cf);
  Py_INCREF(se);
  Py_INCREF(sslerr);
  Py_XINCREF(te);
  Py_XSETREF(g_conn_failed, cf);
  Py_XSETREF(g_status_error, se);
  Py_XSETREF(g_ssl_error, sslerr);
  Py_XSETREF(g_timeout_error, te);
  g_shared_openssl = same_openssl(ssl_path, py_version);
  Py_RETURN_NONE;
}

// ssl_context_supported(ctx) -> bool: can Conn use this TlsContext / ssl.SSLContext natively?
PyObject* ssl_context_supported(PyObject*, PyObject* ctx) {
  if (ssl_ctx_of(ctx)) Py_RETURN_TRUE;
  PyErr_Clear();
  Py_RETURN_FALSE;
}

// openssl() -> (OpenSSL_version_num(), OpenSSL_version(OPENSSL_VERSION), shares CPython's _ssl)
PyObject* openssl_info(PyObject*, PyObject*) {
  return Py_BuildValue("(KsO)", static_cast<unsigned long long>(OpenSSL_version_num()),
                       OpenSSL_version(OPENSSL_VERSION), g_shared_openssl ? Py_True : Py_False);
}

PyMethodDef kMethods[] = {
    {"configure", configure, METH_VARARGS,
     "configure(ConnectionFailed, HttpStatusError, SSLError[, TimeoutError[, ssl_module_path, "
     "ssl_openssl_version_number]])"},
    {"ssl_context_supported", ssl_context_supported, METH_O,
     "ssl_context_supported(ctx) -> bool: the context's SSL_CTX can be used natively"},
    {"openssl", openssl_info, METH_NOARGS,
     "openssl() -> (version number, version text, shared with CPython's ssl module)"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_netconn", "Native HTTP/1.1 client connection for asyncio.", -1,
                       kMethods, nullptr, nullptr, nullptr, nullptr};

bool intern(PyObject** slot, const char* s) {
  *slot = PyUnicode_InternFromString(s);
  return *slot != nullptr;
}

}  // namespace

PyMODINIT_FUNC PyInit__netconn(void) {
  if (!intern(&s_create_future, "create_future") || !intern(&s_set_result, "set_result") ||
      !intern(&s_set_exception, "set_exception") || !intern(&s_done, "done") ||
      !intern(&s_add_reader, "add_reader") || !intern(&s_remove_reader, "remove_reader") ||
      !intern(&s_add_writer, "add_writer") || !intern(&s_remove_writer, "remove_writer") ||
      !intern(&s_on_readable, "_on_readable") || !intern(&s_on_writable, "_on_writable") ||
      !intern(&s_options, "options") || !intern(&s_verify_mode, "verify_mode"))
    return nullptr;
  TlsCtxType.tp_dealloc = reinterpret_cast<destructor>(tls_dealloc);
  TlsCtxType.tp_flags = Py_TPFLAGS_DEFAULT;
  TlsCtxType.tp_doc = "An SSL_CTX built by _netconn from PEM material (the linked libssl).";
  TlsCtxType.tp_getset = kTlsGetSet;
  TlsCtxType.tp_init = reinterpret_cast<initproc>(tls_init);
  TlsCtxType.tp_new = PyType_GenericNew;
  if (PyType_Ready(&TlsCtxType) < 0) return nullptr;
  ConnType.tp_dealloc = reinterpret_cast<destructor>(conn_dealloc);
  ConnType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_BASETYPE | Py_TPFLAGS_HAVE_GC;
  ConnType.tp_doc = "One HTTP/1.1 client connection driven by an asyncio loop.";
  ConnType.tp_traverse = reinterpret_cast<traverseproc>(conn_traverse);
  ConnType.tp_clear = reinterpret_cast<inquiry>(conn_clear);
  ConnType.tp_weaklistoffset = offsetof(ConnObject, weakrefs);
  ConnType.tp_methods = kConnMethods;
  ConnType.tp_members = kConnMembers;
  ConnType.tp_getset = kConnGetSet;
  ConnType.tp_init = reinterpret_cast<initproc>(conn_init);
  ConnType.tp_new = conn_new;
  if (PyType_Ready(&ConnType) < 0) return nullptr;
  PoolType.tp_dealloc = reinterpret_cast<destructor>(pool_dealloc);
  PoolType.tp_flags = Py_TPFLAGS_DEFAULT | Py_TPFLAGS_HAVE_GC;
  PoolType.tp_doc = "Keep-alive pool of native connections to one server: request path in C++.";
  PoolType.tp_traverse = reinterpret_cast<traverseproc>(pool_traverse);
  PoolType.tp_clear = reinterpret_cast<inquiry>(pool_clear);
  PoolType.tp_weaklistoffset = offsetof(PoolObject, weakrefs);
  PoolType.tp_methods = kPoolMethods;
  PoolType.tp_members = kPoolMembers;
  PoolType.tp_getset = kPoolGetSet;
  PoolType.tp_init = reinterpret_cast<initproc>(pool_init);
  PoolType.tp_new = pool_new;
  if (PyType_Ready(&PoolType) < 0) return nullptr;
  PyObject* m = PyModule_Create(&kModule);
  if (!m) return nullptr;
  Py_INCREF(&ConnType);
  if (PyModule_AddObject(m, "Conn", reinterpret_cast<PyObject*>(&ConnType)) < 0) {
    Py_DECREF(&ConnType);
    Py_DECREF(m);
    return nullptr;
  }
  Py_INCREF(&PoolType);
  if (PyModule_AddObject(m, "Pool", reinterpret_cast<PyObject*>(&PoolType)) < 0) {
    Py_DECREF(&PoolType);
    Py_DECREF(m);
    return nullptr;
  }
  Py_INCREF(&TlsCtxType);
  if (PyModule_AddObject(m, "TlsContext", reinterpret_cast<PyObject*>(&TlsCtxType)) < 0) {
    Py_DECREF(&TlsCtxType);
    Py_DECREF(m);
    return nullptr;
  }
  return m;
}
