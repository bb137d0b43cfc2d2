// store.h -- rendezvous key/value stores (gloo/rendezvous/store.h).
//
// The stores carry only bootstrap metadata (endpoint descriptions, IPC
// handles, flag-word indices); nothing on the data path touches them.
//   HashStore     in-process map, ranks are threads  (gloo/rendezvous/hash_store.h:20)
//   FileStore     one file per key in a shared dir   (gloo/rendezvous/file_store.h:19)
//   PrefixStore   key namespacing                    (gloo/rendezvous/prefix_store.h)
//   CallbackStore set/get supplied by the caller (e.g. torch.distributed's
//                 TCPStore bridged from Python)
#pragma once

#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gloo_amd/glx.h"

namespace gloo {
namespace rendezvous {

class Store {
 public:
  virtual ~Store() = default;

  virtual void set(const std::string& key, const std::vector<char>& data) = 0;

  // Non-blocking lookup; false if the key does not exist yet.
  virtual bool tryGet(const std::string& key, std::vector<char>* out) = 0;

  // Blocking lookup (gloo Store::get semantics); throws TimeoutException.
  virtual std::vector<char> get(const std::string& key,
                                std::chrono::milliseconds timeout);

  void wait(const std::vector<std::string>& keys,
            std::chrono::milliseconds timeout);
};

class HashStore : public Store {
 public:
  void set(const std::string& key, const std::vector<char>& data) override;
  bool tryGet(const std::string& key, std::vector<char>* out) override;
  std::vector<char> get(const std::string& key,
                        std::chrono::milliseconds timeout) override;

 private:
  std::mutex m_;
  std::condition_variable cv_;
  std::map<std::string, std::vector<char>> map_;
};

class FileStore : public Store {
 public:
  explicit FileStore(const std::string& path);
  void set(const std::string& key, const std::vector<char>& data) override;
  bool tryGet(const std::string& key, std::vector<char>* out) override;

 private:
  std::string pathFor(const std::string& key) const;
  std::string path_;
};

class PrefixStore : public Store {
 public:
  PrefixStore(const std::string& prefix, std::shared_ptr<Store> base)
      : prefix_(prefix), base_(std::move(base)) {}
  void set(const std::string& key, const std::vector<char>& data) override {
    base_->set(prefix_ + "/" + key, data);
  }
  bool tryGet(const std::string& key, std::vector<char>* out) override {
    return base_->tryGet(prefix_ + "/" + key, out);
  }
  std::vector<char> get(const std::string& key,
                        std::chrono::milliseconds timeout) override {
    return base_->get(prefix_ + "/" + key, timeout);
  }

 private:
  std::string prefix_;
  std::shared_ptr<Store> base_;
};

class CallbackStore : public Store {
 public:
  CallbackStore(glx_store_set_fn set_fn, glx_store_get_fn get_fn, void* user)
      : set_(set_fn), get_(get_fn), user_(user) {}
  void set(const std::string& key, const std::vector<char>& data) override;
  bool tryGet(const std::string& key, std::vector<char>* out) override;

 private:
  glx_store_set_fn set_;
  glx_store_get_fn get_;
  void* user_;
};

}  // namespace rendezvous
}  // namespace gloo
