// jit.hip -- hiprtc front-end: compile, cache (memory + disk) and load specialised kernels.
#include "jit.h"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <sstream>
#include <unordered_map>
#include <vector>

#include "jit_src.inc"

namespace bqg {
namespace {

struct Rtc {
  decltype(&hiprtcCreateProgram) create = nullptr;
  decltype(&hiprtcCompileProgram) compile = nullptr;
  decltype(&hiprtcGetProgramLogSize) log_size = nullptr;
  decltype(&hiprtcGetProgramLog) log = nullptr;
  decltype(&hiprtcGetCodeSize) code_size = nullptr;
  decltype(&hiprtcGetCode) code = nullptr;
  decltype(&hiprtcDestroyProgram) destroy = nullptr;
  bool ok = false;

  Rtc() {
    void* h = dlopen("libhiprtc.so.7", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("libhiprtc.so.7", RTLD_NOW);
    if (!h) h = dlopen("/opt/rocm/lib/libhiprtc.so.7", RTLD_NOW);
    if (!h) return;
    create = (decltype(create))dlsym(h, "hiprtcCreateProgram");
    compile = (decltype(compile))dlsym(h, "hiprtcCompileProgram");
    log_size = (decltype(log_size))dlsym(h, "hiprtcGetProgramLogSize");
    log = (decltype(log))dlsym(h, "hiprtcGetProgramLog");
    code_size = (decltype(code_size))dlsym(h, "hiprtcGetCodeSize");
    code = (decltype(code))dlsym(h, "hiprtcGetCode");
    destroy = (decltype(destroy))dlsym(h, "hiprtcDestroyProgram");
    ok = create && compile && log_size && log && code_size && code && destroy;
  }
};

// hiprtc has no libc headers: the public header's <stddef.h> / <stdint.h> resolve to these
const char* kStddef = "#pragma once\n";
const char* kStdint =
    "#pragma once\n"
    "typedef __hip_internal::int8_t int8_t; typedef __hip_internal::uint8_t uint8_t;\n"
    "typedef __hip_internal::int16_t int16_t; typedef __hip_internal::uint16_t uint16_t;\n"
    "typedef __hip_internal::int32_t int32_t; typedef __hip_internal::uint32_t uint32_t;\n"
    "typedef __hip_internal::int64_t int64_t; typedef __hip_internal::uint64_t uint64_t;\n";

const char* kOptions[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-munsafe-fp-atomics",
                          "-ffp-contract=fast-honor-pragmas"};

uint64_t fnv1a(const std::string& s, uint64_t h = 1469598103934665603ull) {
  for (unsigned char ch : s) h = (h ^ ch) * 1099511628211ull;
  return h;
}

std::string cache_dir() {
  std::string d;
  if (const char* e = getenv("BQGPU_JIT_CACHE")) d = e;
  else if (const char* x = getenv("XDG_CACHE_HOME")) d = std::string(x) + "/bqgpu-jit";
  else if (const char* h = getenv("HOME")) d = std::string(h) + "/.cache/bqgpu-jit";
  else d = "/tmp/bqgpu-jit-" + std::to_string(getuid());
  return d;
}

void mkdirs(const std::string& d) {
  for (size_t i = 1; i <= d.size(); ++i)
    if (i == d.size() || d[i] == '/') mkdir(d.substr(0, i).c_str(), 0755);
}

bool read_file(const std::string& path, std::vector<char>& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f) return false;
  out.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
  return !out.empty();
}

void write_file(const std::string& path, const std::vector<char>& data) {
  const std::string tmp = path + ".tmp." + std::to_string(getpid());
  {
    std::ofstream f(tmp, std::ios::binary);
    if (!f) return;
    f.write(data.data(), (std::streamsize)data.size());
  }
  if (rename(tmp.c_str(), path.c_str()) != 0) unlink(tmp.c_str());
}

struct JitState {
  std::mutex mu;
  Rtc* rtc = nullptr;
  bool tried = false;
  std::map<std::string, hipFunction_t> fns;  // device:kernel:hash -> function (nullptr = failed)
  // per-query front cache (jit_function_for): binary shape key -> function, so a repeated query
  // shape costs one hash lookup instead of formatting and hashing its prologue
  std::unordered_map<std::string, hipFunction_t> by_shape;

  bool compile(const std::string& src, std::vector<char>& code) {
    if (!tried) {
      tried = true;
      rtc = new Rtc();
    }
    if (!rtc->ok) return false;
    std::vector<const char*> names(kJitHeaderNames, kJitHeaderNames + kJitHeaderCount);
    std::vector<const char*> texts(kJitHeaderTexts, kJitHeaderTexts + kJitHeaderCount);
    names.push_back("stddef.h");
    texts.push_back(kStddef);
    names.push_back("stdint.h");
    texts.push_back(kStdint);
    hiprtcProgram prog;
    if (rtc->create(&prog, src.c_str(), "bq_jit.hip", (int)names.size(), texts.data(), names.data()) !=
        HIPRTC_SUCCESS)
      return false;
    const hiprtcResult r = rtc->compile(prog, (int)(sizeof(kOptions) / sizeof(kOptions[0])), kOptions);
    bool ok = r == HIPRTC_SUCCESS;
    if (!ok && getenv("BQGPU_JIT_VERBOSE")) {
      size_t n = 0;
      rtc->log_size(prog, &n);
      std::string log(n, ' ');
      rtc->log(prog, &log[0]);
      fprintf(stderr, "bqgpu jit: compile failed:\n%s\n", log.c_str());
    }
    if (ok) {
      size_t n = 0;
      ok = rtc->code_size(prog, &n) == HIPRTC_SUCCESS && n > 0;
      if (ok) {
        code.resize(n);
        ok = rtc->code(prog, code.data()) == HIPRTC_SUCCESS;
      }
    }
    rtc->destroy(&prog);
    return ok;
  }
};

JitState& state() {
  static JitState* s = new JitState();  // never destroyed: modules live as long as the process
  return *s;
}

}  // namespace

namespace {

// Every ScanParams field the specialisation reads, in prologue order: f(array, index, field,
// value, suffix) -- "p.cols[0].dtype=3;" is ("p.cols", 0, "dtype", 3, ""), "p.ncols=2;" is
// ("p", -1, "ncols", 2, ""), "p.sum_conv[1]=0;" is ("p.sum_conv", 1, nullptr, 0, "").  The
// prologue text and the per-query cache key below are both built from this one list.
template <class F>
void spec_fields(const ScanParams& p, F&& f) {
  f("p", -1, "ncols", p.ncols, "");
  for (int c = 0; c < p.ncols; ++c) {
    f("p.cols", c, "dtype", p.cols[c].dtype, "");
    f("p.cols", c, "lg", p.cols[c].lg, "");
    f("p.cols", c, "enc", p.cols[c].enc, "");
  }
  f("p", -1, "nterms", p.nterms, "");
  for (int t = 0; t < p.nterms; ++t) {
    const DevTerm& tm = p.terms[t];
    f("p.terms", t, "col", tm.col, "");
    f("p.terms", t, "op", tm.op, "");
    f("p.terms", t, "is_float", tm.is_float, "");
    if ((tm.op == BQG_T_IN || tm.op == BQG_T_NIN) && tm.nvals <= 8) f("p.terms", t, "nvals", tm.nvals, "");
  }
  f("p", -1, "nkeys", p.nkeys, "");
  for (int k = 0; k < p.nkeys; ++k) {
    const DevKey& key = p.keys[k];
    f("p.keys", k, "col", key.col, "");
    f("p.keys", k, "is_float", key.is_float, "");
    if (key.stride == 1) f("p.keys", k, "stride", 1, "ull");
  }
  f("p", -1, "nsum", p.nsum, "");
  for (int i = 0; i < p.nsum && i < kMaxSums; ++i) {
    f("p.sum_is_float", i, nullptr, p.sum_is_float[i], "");
    f("p.sum_conv", i, nullptr, p.sum_conv[i], "");
    f("p.sum_centered", i, nullptr, p.sum_centered[i], "");
  }
  f("p", -1, "mask_col", p.mask_col, "");
  f("p", -1, "hash", p.hash, "");
}

}  // namespace

std::string jit_spec(const ScanParams& p) {
  std::ostringstream s;
  s << "#define BQ_NC " << p.ncols << "\n#define BQ_SPEC ";
  spec_fields(p, [&](const char* arr, int idx, const char* field, long long v, const char* sfx) {
    s << arr;
    if (idx >= 0) s << "[" << idx << "]";
    if (field) s << "." << field;
    s << "=" << v << sfx << ";";
  });
  s << "\n";
  return s.str();
}

hipFunction_t jit_function_for(const char* kernel, const ScanParams& p, const std::string& extra) {
  // the key: device, kernel, extra defines, then (field, value) for every specialised field --
  // the field names' addresses mark which conditional fields are present
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::string key;
  key.reserve(512 + extra.size());
  key.append((const char*)&dev, sizeof(dev));
  key.append(kernel);
  key.push_back('\0');
  key.append(extra);
  key.push_back('\0');
  spec_fields(p, [&](const char* arr, int, const char* field, long long v, const char*) {
    const void* tag[2] = {arr, field};
    key.append((const char*)tag, sizeof(tag));
    key.append((const char*)&v, sizeof(v));
  });
  JitState& js = state();
  {
    std::lock_guard<std::mutex> lk(js.mu);
    auto it = js.by_shape.find(key);
    if (it != js.by_shape.end()) return it->second;
  }
  hipFunction_t fn = jit_function(kernel, jit_spec(p) + extra);
  std::lock_guard<std::mutex> lk(js.mu);
  js.by_shape.emplace(std::move(key), fn);
  return fn;
}

hipFunction_t jit_function(const char* kernel, const std::string& spec) {
  JitState& js = state();
  std::lock_guard<std::mutex> lk(js.mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const std::string src = spec + "#include \"jit_kernels.h\"\n";
  // the embedded headers and options hash once per process (~100 KB of text), the spec per call
  static const uint64_t kSourceHash = [] {
    uint64_t hh = 1469598103934665603ull;
    for (int i = 0; i < kJitHeaderCount; ++i) hh = fnv1a(kJitHeaderTexts[i], hh);
    for (const char* o : kOptions) hh = fnv1a(o, hh);
    return hh;
  }();
  const uint64_t h = fnv1a(src, kSourceHash);
  char hex[17];
  snprintf(hex, sizeof(hex), "%016llx", (unsigned long long)h);
  const std::string key = std::to_string(dev) + ":" + kernel + ":" + hex;
  auto it = js.fns.find(key);
  if (it != js.fns.end()) return it->second;
  hipFunction_t fn = nullptr;
  std::vector<char> code;
  const std::string dir = cache_dir();
  const std::string path = dir + "/" + hex + ".hsaco";
  if (!read_file(path, code)) {
    if (js.compile(src, code)) {
      mkdirs(dir);
      write_file(path, code);
    } else {
      code.clear();
    }
  }
  if (!code.empty()) {
    hipModule_t mod = nullptr;
    if (hipModuleLoadData(&mod, code.data()) == hipSuccess) {
      if (hipModuleGetFunction(&fn, mod, kernel) != hipSuccess) fn = nullptr;
    } else {
      (void)hipGetLastError();
    }
  }
  js.fns[key] = fn;
  return fn;
}

}  // namespace bqg

// Test hook (not part of include/bqgpu.h): compile one specialised private scan for the
// prologue `spec` without loading it (no GPU needed).  0 = compiled, 1 = hiprtc missing,
// 2 = compile error (log on stderr).
extern "C" int bqg_internal_jit_compile_check(const char* spec) {
  using namespace bqg;
  JitState& js = state();
  std::lock_guard<std::mutex> lk(js.mu);
  std::vector<char> code;
  setenv("BQGPU_JIT_VERBOSE", "1", 0);
  if (js.compile(std::string(spec) + "#include \"jit_kernels.h\"\n", code)) return 0;
  return js.rtc && js.rtc->ok ? 2 : 1;
}
