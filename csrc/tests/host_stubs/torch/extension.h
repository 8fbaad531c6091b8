// Host-only stand-in for the parts of <torch/extension.h> (ATen + pybind11) that the native
// runtime (csrc/comm/rccl_engine.h, csrc/runtime/stage_runner.cpp) uses, so those sources
// build with plain g++ under -fsanitize=address,undefined (csrc/tests/host_asan_test.cpp).
// Nothing here talks to Python: py::object holds a C++ pointer, py::function a
// std::function, py::list / py::dict are plain containers.
#pragma once
#include <any>
#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

namespace fake_torch {
inline void cat_into(std::ostringstream&) {}
template <typename T, typename... R>
void cat_into(std::ostringstream& o, const T& v, const R&... r) {
  o << v;
  cat_into(o, r...);
}
template <typename... A>
std::string cat(const A&... a) {
  std::ostringstream o;
  cat_into(o, a...);
  return o.str();
}
}  // namespace fake_torch

#define TORCH_CHECK(cond, ...)                                                   \
  do {                                                                           \
    if (!(cond)) throw std::runtime_error(::fake_torch::cat("", ##__VA_ARGS__)); \
  } while (0)

namespace torch {
enum ScalarType { kUInt8 = 0, kInt32 = 3, kInt64 = 4, kFloat16 = 5, kFloat32 = 6, kFloat64 = 7, kBFloat16 = 15 };
inline std::ostream& operator<<(std::ostream& o, ScalarType t) { return o << "ScalarType(" << (int)t << ")"; }
struct Storage {
  void* p;
  void* data_ptr() const { return p; }
};
// a host buffer that claims to be a contiguous GPU tensor
struct Tensor {
  void* ptr = nullptr;
  int64_t n = 0;
  ScalarType t = kFloat32;
  bool cuda = true;
  bool is_cuda() const { return cuda; }
  bool is_contiguous() const { return true; }
  ScalarType scalar_type() const { return t; }
  int64_t numel() const { return n; }
  void* data_ptr() const { return ptr; }
  Storage storage() const { return Storage{ptr}; }
};
}  // namespace torch

namespace pybind11 {
struct object {
  std::shared_ptr<void> holder;   // keeps the pointee alive like a Python reference
  void* p = nullptr;
  object() = default;
  template <typename T>
  static object of(std::shared_ptr<T> sp) {
    object o;
    o.p = sp.get();
    o.holder = std::move(sp);
    return o;
  }
  template <typename T>
  T cast() const {
    static_assert(std::is_pointer<T>::value, "fake py::object casts to pointers only");
    return static_cast<T>(p);
  }
};
struct function {
  std::function<void()> f;
  function() = default;
  explicit function(std::function<void()> g) : f(std::move(g)) {}
  void operator()() const { f(); }
};
struct bytes : std::string {
  bytes(const char* d, size_t n) : std::string(d, n) {}
  explicit bytes(std::string s) : std::string(std::move(s)) {}
};
struct handle_any {
  std::any v;
  template <typename T>
  handle_any& operator=(T x) {
    v = std::move(x);
    return *this;
  }
};
inline handle_any cast(std::vector<int> v) {
  handle_any h;
  h.v = std::move(v);
  return h;
}
struct dict {
  std::shared_ptr<std::map<std::string, handle_any>> m = std::make_shared<std::map<std::string, handle_any>>();
  handle_any& operator[](const char* k) { return (*m)[k]; }
  bool contains(const std::string& k) const { return m->count(k) != 0; }
  template <typename T>
  T get(const std::string& k) const { return std::any_cast<T>(m->at(k).v); }
};
struct list {
  std::vector<dict> items;
  void append(const dict& d) { items.push_back(d); }
  size_t size() const { return items.size(); }
};
struct gil_scoped_release {};
struct gil_scoped_acquire {};
struct module {
  std::map<std::string, handle_any> attrs;
  template <typename... A>
  module& def(A&&...) { return *this; }
  handle_any& attr(const char* k) { return attrs[k]; }
};
template <typename... A>
struct init {};
struct arg {
  explicit arg(const char*) {}
  template <typename T>
  arg& operator=(const T&) { return *this; }
};
template <typename C>
struct class_ {
  class_(module&, const char*) {}
  template <typename... A>
  class_& def(A&&...) { return *this; }
  template <typename... A>
  class_& def_static(A&&...) { return *this; }
  template <typename... A>
  class_& def_property_readonly(A&&...) { return *this; }
};
}  // namespace pybind11
