// store.cc -- rendezvous stores.  See store.h.
#include "store.h"

#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <thread>

#include "common.h"

namespace gloo {
namespace rendezvous {

std::vector<char> Store::get(const std::string& key,
                             std::chrono::milliseconds timeout) {
  const auto deadline = std::chrono::steady_clock::now() + timeout;
  auto sleep = std::chrono::microseconds(50);
  std::vector<char> out;
  for (;;) {
    if (tryGet(key, &out)) return out;
    if (std::chrono::steady_clock::now() > deadline) {
      GLX_THROW_TIMEOUT("Timed out waiting for store key '", key, "' after ",
                        timeout.count(), " ms");
    }
    std::this_thread::sleep_for(sleep);
    if (sleep < std::chrono::milliseconds(5)) sleep *= 2;
  }
}

void Store::wait(const std::vector<std::string>& keys,
                 std::chrono::milliseconds timeout) {
  for (const auto& k : keys) get(k, timeout);
}

// ---- HashStore ------------------------------------------------------------

void HashStore::set(const std::string& key, const std::vector<char>& data) {
  {
    std::lock_guard<std::mutex> g(m_);
    map_[key] = data;
  }
  cv_.notify_all();
}

bool HashStore::tryGet(const std::string& key, std::vector<char>* out) {
  std::lock_guard<std::mutex> g(m_);
  auto it = map_.find(key);
  if (it == map_.end()) return false;
  *out = it->second;
  return true;
}

std::vector<char> HashStore::get(const std::string& key,
                                 std::chrono::milliseconds timeout) {
  std::unique_lock<std::mutex> g(m_);
  bool ok = cv_.wait_for(g, timeout, [&] { return map_.count(key) != 0; });
  if (!ok) {
    GLX_THROW_TIMEOUT("Timed out waiting for store key '", key, "' after ",
                      timeout.count(), " ms");
  }
  return map_[key];
}

// ---- FileStore ------------------------------------------------------------

FileStore::FileStore(const std::string& path) : path_(path) {
  // mkdir -p
  std::string cur;
  for (size_t i = 0; i <= path.size(); i++) {
    if (i == path.size() || path[i] == '/') {
      if (!cur.empty() && ::mkdir(cur.c_str(), 0700) != 0 && errno != EEXIST) {
        GLX_THROW_IO("FileStore: mkdir ", cur, " failed: ", strerror(errno));
      }
    }
    if (i < path.size()) cur.push_back(path[i]);
  }
}

std::string FileStore::pathFor(const std::string& key) const {
  static const char* hex = "0123456789abcdef";
  std::string name;
  for (unsigned char c : key) {
    if (isalnum(c) || c == '_' || c == '-' || c == '.') {
      name.push_back((char)c);
    } else {
      name.push_back('%');
      name.push_back(hex[c >> 4]);
      name.push_back(hex[c & 15]);
    }
  }
  return path_ + "/" + name;
}

void FileStore::set(const std::string& key, const std::vector<char>& data) {
  const std::string final_path = pathFor(key);
  const std::string tmp = final_path + ".tmp." + std::to_string(::getpid());
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (f == nullptr) GLX_THROW_IO("FileStore: open ", tmp, ": ", strerror(errno));
  size_t w = data.empty() ? 0 : std::fwrite(data.data(), 1, data.size(), f);
  std::fflush(f);
  ::fsync(fileno(f));
  std::fclose(f);
  if (w != data.size()) GLX_THROW_IO("FileStore: short write to ", tmp);
  // rename is atomic: readers see the whole value or nothing
  if (::rename(tmp.c_str(), final_path.c_str()) != 0) {
    GLX_THROW_IO("FileStore: rename ", tmp, ": ", strerror(errno));
  }
}

bool FileStore::tryGet(const std::string& key, std::vector<char>* out) {
  FILE* f = std::fopen(pathFor(key).c_str(), "rb");
  if (f == nullptr) return false;
  out->clear();
  char buf[4096];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) out->insert(out->end(), buf, buf + n);
  std::fclose(f);
  return true;
}

// ---- CallbackStore --------------------------------------------------------

void CallbackStore::set(const std::string& key, const std::vector<char>& data) {
  int rc = set_(user_, key.c_str(), data.data(), data.size());
  if (rc != 0) GLX_THROW_IO("CallbackStore: set('", key, "') failed rc=", rc);
}

bool CallbackStore::tryGet(const std::string& key, std::vector<char>* out) {
  std::vector<char> buf(256);
  int64_t n = get_(user_, key.c_str(), buf.data(), buf.size());
  if (n == -2) GLX_THROW_IO("CallbackStore: key '", key, "' will never be set");
  if (n < 0) return false;
  if ((size_t)n > buf.size()) {
    buf.resize((size_t)n);
    n = get_(user_, key.c_str(), buf.data(), buf.size());
    if (n == -2) GLX_THROW_IO("CallbackStore: key '", key, "' will never be set");
    if (n < 0) return false;
  }
  buf.resize((size_t)n);
  *out = std::move(buf);
  return true;
}

}  // namespace rendezvous
}  // namespace gloo
