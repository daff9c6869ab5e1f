// gm_sdbus.cpp — the two systemd D-Bus calls gpumounter needs, spoken directly on the socket.
//
// On systemd-cgroup-driver nodes the container's cgroup is a transient systemd scope
// (cri-containerd-<id>.scope, crio-<id>.scope, docker-<id>.scope). systemd owns the device policy
// of that unit (its DeviceAllow= list) and re-applies it whenever it re-realises the unit
// (daemon-reload, unit property changes): on cgroup v1 by rewriting devices.deny/devices.allow,
// on cgroup v2 by attaching a freshly generated device program. A rule gpumounter wrote behind
// systemd's back is lost at that moment. Recording the hot-mounted nodes in the unit's own
// DeviceAllow= (SetUnitProperties, runtime) makes systemd itself keep them.
//
// The reference never faced this (cgroup v1 + cgroupfs driver only: reference
// pkg/util/cgroup/cgroup.go:78-118). No libdbus / sd-bus dependency: the worker image stays
// minimal, and a few hundred lines of marshalling cover the fixed signatures used here.
#include "gm_host.h"

#include <errno.h>
#include <poll.h>
#include <stdio.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <time.h>
#include <unistd.h>

#include <string>
#include <vector>

namespace {

constexpr int kTimeoutMs = 5000;
constexpr uint8_t kMethodCall = 1, kMethodReturn = 2, kError = 3;
constexpr uint8_t kFieldPath = 1, kFieldInterface = 2, kFieldMember = 3, kFieldErrorName = 4,
                  kFieldReplySerial = 5, kFieldDestination = 6, kFieldSignature = 8;

// ------------------------------------------------------------------ marshalling (little endian)
struct Writer {
  std::string b;
  void align(size_t n) {
    while (b.size() % n) b.push_back('\0');
  }
  void u8(uint8_t v) { b.push_back((char)v); }
  void u32(uint32_t v) {
    align(4);
    b.append(reinterpret_cast<const char*>(&v), 4);
  }
  void str(const std::string& s) {  // 's' and 'o'
    u32((uint32_t)s.size());
    b.append(s);
    b.push_back('\0');
  }
  void sig(const std::string& s) {  // 'g'
    u8((uint8_t)s.size());
    b.append(s);
    b.push_back('\0');
  }
  // Arrays: length placeholder, padding to the element alignment, elements, patched length.
  size_t array_begin(size_t elem_align, size_t* start) {
    u32(0);
    size_t len_at = b.size() - 4;
    align(elem_align);
    *start = b.size();
    return len_at;
  }
  void array_end(size_t len_at, size_t start) {
    uint32_t len = (uint32_t)(b.size() - start);
    memcpy(&b[len_at], &len, 4);
  }
};

struct Reader {
  const std::string& b;
  size_t p;
  bool ok = true;
  Reader(const std::string& buf, size_t pos) : b(buf), p(pos) {}
  void align(size_t n) { p = (p + n - 1) / n * n; }
  bool need(size_t n) {
    if (p + n > b.size()) ok = false;
    return ok;
  }
  uint8_t u8() {
    if (!need(1)) return 0;
    return (uint8_t)b[p++];
  }
  uint32_t u32() {
    align(4);
    if (!need(4)) return 0;
    uint32_t v;
    memcpy(&v, &b[p], 4);
    p += 4;
    return v;
  }
  std::string str() {
    uint32_t n = u32();
    if (!need((size_t)n + 1)) return "";
    std::string s = b.substr(p, n);
    p += n + 1;
    return s;
  }
  std::string sig() {
    uint8_t n = u8();
    if (!need((size_t)n + 1)) return "";
    std::string s = b.substr(p, n);
    p += n + 1;
    return s;
  }
};

struct Field {
  uint8_t code;
  char type;  // 's', 'o', 'g', 'u'
  std::string s;
  uint32_t u;
};

std::string build_message(uint32_t serial, const std::vector<Field>& fields, const std::string& body,
                          uint8_t flags = 0) {
  Writer w;
  w.u8('l');
  w.u8(kMethodCall);
  w.u8(flags);
  w.u8(1);
  w.u32((uint32_t)body.size());
  w.u32(serial);
  size_t start;
  size_t len_at = w.array_begin(8, &start);
  for (const Field& f : fields) {
    w.align(8);
    w.u8(f.code);
    w.sig(std::string(1, f.type));
    if (f.type == 'u') w.u32(f.u);
    else if (f.type == 'g') w.sig(f.s);
    else w.str(f.s);
  }
  w.array_end(len_at, start);
  w.align(8);
  w.b.append(body);
  return w.b;
}

struct Message {
  uint8_t type = 0;
  uint32_t reply_serial = 0;
  std::string error_name, signature, raw;
  size_t body_at = 0;
};

// ------------------------------------------------------------------ socket I/O
int64_t now_ms() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

int wait_fd(int fd, short ev, int64_t deadline) {
  for (;;) {
    int left = (int)(deadline - now_ms());
    if (left <= 0) return -ETIMEDOUT;
    struct pollfd p = {fd, ev, 0};
    int r = poll(&p, 1, left);
    if (r > 0) return 0;
    if (r == 0) return -ETIMEDOUT;
    if (errno != EINTR) return -errno;
  }
}

int send_all(int fd, const char* p, size_t n, int64_t deadline) {
  while (n) {
    ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        int e = wait_fd(fd, POLLOUT, deadline);
        if (e < 0) return e;
        continue;
      }
      return -errno;
    }
    p += w;
    n -= (size_t)w;
  }
  return 0;
}

int recv_exact(int fd, std::string* out, size_t n, int64_t deadline) {
  size_t have = out->size();
  out->resize(have + n);
  size_t got = 0;
  while (got < n) {
    int e = wait_fd(fd, POLLIN, deadline);
    if (e < 0) return e;
    ssize_t r = recv(fd, &(*out)[have + got], n - got, 0);
    if (r == 0) return -ECONNRESET;
    if (r < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;
      return -errno;
    }
    got += (size_t)r;
  }
  return 0;
}

int recv_line(int fd, std::string* line, int64_t deadline) {
  line->clear();
  while (line->size() < 512) {
    std::string c;
    int e = recv_exact(fd, &c, 1, deadline);
    if (e < 0) return e;
    line->append(c);
    if (line->size() >= 2 && line->compare(line->size() - 2, 2, "\r\n") == 0) return 0;
  }
  return -EPROTO;
}

int read_message(int fd, Message* m, int64_t deadline) {
  std::string& b = m->raw;
  b.clear();
  int e = recv_exact(fd, &b, 16, deadline);
  if (e < 0) return e;
  if (b[0] != 'l' || b[3] != 1) return -EPROTO;  // systemd on little-endian hosts sends 'l'
  uint32_t body_len, fields_len;
  memcpy(&body_len, &b[4], 4);
  memcpy(&fields_len, &b[12], 4);
  if (fields_len > (1u << 20) || body_len > (64u << 20)) return -EPROTO;
  size_t hdr_end = 16 + fields_len;
  size_t body_at = (hdr_end + 7) / 8 * 8;
  e = recv_exact(fd, &b, body_at - 16 + body_len, deadline);
  if (e < 0) return e;
  m->type = (uint8_t)b[1];
  m->body_at = body_at;
  m->reply_serial = 0;
  m->error_name.clear();
  m->signature.clear();
  Reader r(b, 16);
  while (r.ok && r.p < hdr_end) {
    r.align(8);
    if (r.p >= hdr_end) break;
    uint8_t code = r.u8();
    std::string t = r.sig();
    if (t == "u") {
      uint32_t v = r.u32();
      if (code == kFieldReplySerial) m->reply_serial = v;
    } else if (t == "s" || t == "o") {
      std::string v = r.str();
      if (code == kFieldErrorName) m->error_name = v;
    } else if (t == "g") {
      std::string v = r.sig();
      if (code == kFieldSignature) m->signature = v;
    } else {
      return -EPROTO;  // no other header field types are sent by systemd / dbus-daemon
    }
  }
  return r.ok ? 0 : -EPROTO;
}

void set_err(char* err, int cap, const std::string& s) {
  if (err && cap > 0) snprintf(err, (size_t)cap, "%s", s.c_str());
}

// ------------------------------------------------------------------ connection
struct Conn {
  int fd = -1;
  bool bus = false;  // true: message bus (Hello + destination), false: systemd's private socket
  uint32_t serial = 0;
  int64_t deadline = 0;
  ~Conn() {
    if (fd >= 0) close(fd);
  }

  int open_socket(const char* path) {
    deadline = now_ms() + kTimeoutMs;
    fd = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC | SOCK_NONBLOCK, 0);
    if (fd < 0) return -errno;
    struct sockaddr_un a;
    memset(&a, 0, sizeof(a));
    a.sun_family = AF_UNIX;
    if (strlen(path) >= sizeof(a.sun_path)) return -ENAMETOOLONG;
    strcpy(a.sun_path, path);
    if (connect(fd, reinterpret_cast<struct sockaddr*>(&a), sizeof(a)) < 0) {
      if (errno != EINPROGRESS && errno != EAGAIN) return -errno;
      int e = wait_fd(fd, POLLOUT, deadline);
      if (e < 0) return e;
    }
    // SASL EXTERNAL with our uid (the kernel vouches for it via SO_PEERCRED).
    std::string uid = std::to_string(getuid()), hex;
    for (char c : uid) {
      char h[3];
      snprintf(h, sizeof(h), "%02x", (unsigned char)c);
      hex += h;
    }
    std::string auth = std::string(1, '\0') + "AUTH EXTERNAL " + hex + "\r\n";
    int e = send_all(fd, auth.data(), auth.size(), deadline);
    if (e < 0) return e;
    std::string line;
    e = recv_line(fd, &line, deadline);
    if (e < 0) return e;
    if (line.compare(0, 3, "OK ") != 0) return -EACCES;
    e = send_all(fd, "BEGIN\r\n", 7, deadline);
    if (e < 0) return e;
    return 0;
  }

  // Sends a method call and waits for its reply (signals and unrelated replies are skipped).
  int call(const std::string& dest, const std::string& path, const std::string& iface,
           const std::string& member, const std::string& signature, const std::string& body,
           Message* reply, char* err, int errcap) {
    std::vector<Field> f = {{kFieldPath, 'o', path, 0},
                            {kFieldInterface, 's', iface, 0},
                            {kFieldMember, 's', member, 0}};
    if (!dest.empty()) f.push_back({kFieldDestination, 's', dest, 0});
    if (!signature.empty()) f.push_back({kFieldSignature, 'g', signature, 0});
    const uint32_t my = ++serial;
    std::string msg = build_message(my, f, body);
    int e = send_all(fd, msg.data(), msg.size(), deadline);
    if (e < 0) return e;
    for (;;) {
      e = read_message(fd, reply, deadline);
      if (e < 0) return e;
      if ((reply->type == kMethodReturn || reply->type == kError) && reply->reply_serial == my)
        break;
    }
    if (reply->type == kError) {
      std::string text = reply->error_name;
      if (reply->signature.size() && reply->signature[0] == 's') {
        Reader r(reply->raw, reply->body_at);
        std::string m = r.str();
        if (r.ok) text += ": " + m;
      }
      set_err(err, errcap, text);
      return -EPROTO;
    }
    return 0;
  }

  int hello(char* err, int errcap) {
    Message m;
    return call("org.freedesktop.DBus", "/org/freedesktop/DBus", "org.freedesktop.DBus", "Hello",
                "", "", &m, err, errcap);
  }
};

int connect_bus(Conn* c, const char* bus_path, char* err, int errcap) {
  if (!bus_path || !*bus_path) return -EINVAL;
  int e = c->open_socket(bus_path);
  if (e < 0) {
    set_err(err, errcap, std::string("connect ") + bus_path + ": " + strerror(-e));
    return e;
  }
  // systemd's private socket is peer-to-peer; anything else is taken to be a message bus, which
  // must see Hello first. A peer that does not know Hello is a direct connection after all.
  c->bus = strstr(bus_path, "systemd/private") == nullptr;
  if (!c->bus) return 0;
  char herr[256] = {0};
  e = c->hello(herr, sizeof(herr));
  if (e == -EPROTO && strstr(herr, "org.freedesktop.DBus.Error.UnknownMethod") == herr) {
    c->bus = false;
    return 0;
  }
  if (e < 0) set_err(err, errcap, herr);
  return e;
}

std::string unit_object_path(const std::string& unit) {
  // sd_bus_path_encode("/org/freedesktop/systemd1/unit", unit): every byte outside [A-Za-z0-9]
  // (and a leading digit) becomes _xx.
  std::string out = "/org/freedesktop/systemd1/unit/";
  if (unit.empty()) return out + "_";
  for (size_t i = 0; i < unit.size(); ++i) {
    unsigned char ch = (unsigned char)unit[i];
    bool alpha = (ch >= 'A' && ch <= 'Z') || (ch >= 'a' && ch <= 'z');
    bool digit = ch >= '0' && ch <= '9';
    if (alpha || (digit && i > 0)) {
      out.push_back((char)ch);
    } else {
      char h[4];
      snprintf(h, sizeof(h), "_%02x", ch);
      out += h;
    }
  }
  return out;
}

std::string unit_interface(const std::string& unit) {
  auto ends = [&](const char* s) {
    size_t n = strlen(s);
    return unit.size() >= n && unit.compare(unit.size() - n, n, s) == 0;
  };
  if (ends(".scope")) return "org.freedesktop.systemd1.Scope";
  if (ends(".slice")) return "org.freedesktop.systemd1.Slice";
  if (ends(".socket")) return "org.freedesktop.systemd1.Socket";
  if (ends(".mount")) return "org.freedesktop.systemd1.Mount";
  if (ends(".swap")) return "org.freedesktop.systemd1.Swap";
  return "org.freedesktop.systemd1.Service";
}

}  // namespace

extern "C" {

int gm_sd_unit_path(const char* unit, char* out, int cap) {
  std::string p = unit_object_path(unit ? unit : "");
  if ((int)p.size() + 1 > cap) return -(int)(p.size() + 1);
  memcpy(out, p.c_str(), p.size() + 1);
  return (int)p.size();
}

int gm_sd_get_device_allow(const char* bus_path, const char* unit, char* out, int cap, char* err,
                           int errcap) {
  if (!unit || !out || cap <= 0) return -EINVAL;
  Conn c;
  int e = connect_bus(&c, bus_path, err, errcap);
  if (e < 0) return e;
  Writer body;
  body.str(unit_interface(unit));
  body.str("DeviceAllow");
  Message m;
  e = c.call("org.freedesktop.systemd1", unit_object_path(unit), "org.freedesktop.DBus.Properties",
             "Get", "ss", body.b, &m, err, errcap);
  if (e < 0) return e;
  if (m.signature != "v") {
    set_err(err, errcap, "unexpected reply signature " + m.signature);
    return -EPROTO;
  }
  Reader r(m.raw, m.body_at);
  if (r.sig() != "a(ss)") {
    set_err(err, errcap, "DeviceAllow is not a(ss)");
    return -EPROTO;
  }
  uint32_t len = r.u32();
  r.align(8);
  const size_t end = r.p + len;
  std::string text;
  while (r.ok && r.p < end) {
    r.align(8);
    std::string path = r.str();
    std::string perm = r.str();
    text += path + "\t" + perm + "\n";
  }
  if (!r.ok) return -EPROTO;
  if ((int)text.size() + 1 > cap) return -ENOSPC;
  memcpy(out, text.c_str(), text.size() + 1);
  return (int)text.size();
}

int gm_sd_set_device_allow(const char* bus_path, const char* unit, const char* const* paths,
                           const char* const* perms, int n, int reset, char* err, int errcap) {
  if (!unit || n < 0 || (n > 0 && (!paths || !perms))) return -EINVAL;
  Conn c;
  int e = connect_bus(&c, bus_path, err, errcap);
  if (e < 0) return e;
  // SetUnitProperties(s name, b runtime, a(sv) properties). An empty DeviceAllow array resets
  // the list; properties apply in order, so [reset, entries] replaces it atomically.
  Writer body;
  body.str(unit);
  body.u32(1);  // runtime: /run, gone at reboot (the container's scope is transient anyway)
  size_t props_start;
  size_t props_len = body.array_begin(8, &props_start);
  auto device_allow = [&](int from, int to) {
    body.align(8);
    body.str("DeviceAllow");
    body.sig("a(ss)");
    size_t st;
    size_t la = body.array_begin(8, &st);
    for (int i = from; i < to; ++i) {
      body.align(8);
      body.str(paths[i]);
      body.str(perms[i]);
    }
    body.array_end(la, st);
  };
  if (reset) device_allow(0, 0);
  if (n > 0) device_allow(0, n);
  body.array_end(props_len, props_start);
  Message m;
  return c.call("org.freedesktop.systemd1", "/org/freedesktop/systemd1",
                "org.freedesktop.systemd1.Manager", "SetUnitProperties", "sba(sv)", body.b, &m,
                err, errcap);
}

}  // extern "C"
