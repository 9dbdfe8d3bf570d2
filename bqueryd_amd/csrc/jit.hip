// jit.hip -- hiprtc front-end: compile, cache (memory + disk) and load specialised kernels.
#include "jit.h"

#include <dlfcn.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <mutex>
#include <set>
#include <sstream>
#include <thread>
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
  // shape costs one hash lookup instead of formatting and hashing its prologue (final answers
  // only: a shape whose compile is still queued is looked up again)
  std::unordered_map<std::string, hipFunction_t> by_shape;
  // background compiles (jit_function(..., async)): a cache miss queues the source and the
  // query runs the precompiled generic kernel; the worker thread compiles, writes the disk
  // cache and leaves the code object here, and the next query of that shape loads it (module
  // loads stay on the querying thread, on its device)
  struct Job {
    std::string key, src, path;  // key: kernel:hash (the code object serves every device)
    std::string fkey, kernel;    // the function's key in `fns` and its name, on device `dev`
    int dev;
  };
  std::deque<Job> queue;
  std::set<std::string> pending;                   // keys queued or compiling
  std::map<std::string, std::vector<char>> ready;  // key -> code object (empty: compile failed)
  std::thread worker;
  std::condition_variable cv, cv_idle;
  bool worker_started = false, stopping = false;
  int64_t compiled = 0, failed = 0;

  // hiprtc is dlopen'ed once, by whichever thread needs it first (the background worker, for
  // async queries: the ~1 ms load of hiprtc and comgr stays off the query path)
  std::once_flag rtc_once;
  bool rtc_ok() {
    std::call_once(rtc_once, [this] {
      tried = true;
      rtc = new Rtc();
    });
    return rtc->ok;
  }

  // (the caller holds mu only when it is the synchronous path; hiprtc itself is thread-safe)
  bool compile(const std::string& src, std::vector<char>& code) {
    if (!rtc || !rtc->ok) return false;
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

  void run_worker() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return stopping || !queue.empty(); });
      if (stopping) break;
      Job j = std::move(queue.front());
      queue.pop_front();
      lk.unlock();
      std::vector<char> code;
      // the disk cache first (another process compiled it), else hiprtc
      const bool cached = read_file(j.path, code);
      const bool ok = cached || (rtc_ok() && compile(j.src, code));
      hipFunction_t fn = nullptr;
      if (ok) {
        if (!cached) {
          const std::string dir = j.path.substr(0, j.path.rfind('/'));
          mkdirs(dir);
          write_file(j.path, code);
        }
        // the module load too (~1 ms): the query that next meets this shape just launches it
        if (hipSetDevice(j.dev) == hipSuccess) fn = load(code, j.kernel.c_str());
      }
      lk.lock();
      (ok ? compiled : failed) += 1;
      if (!ok) code.clear();
      fns[j.fkey] = fn;
      ready[j.key] = std::move(code);
      pending.erase(j.key);
      if (pending.empty()) cv_idle.notify_all();
    }
    pending.clear();
    cv_idle.notify_all();
  }

  // (mu held) start the worker on first use; at process exit it finishes the compile in
  // flight and drops the rest (a detached compile racing the runtime's teardown could crash)
  void enqueue(Job j) {
    pending.insert(j.key);
    queue.push_back(std::move(j));
    if (!worker_started) {
      worker_started = true;
      worker = std::thread([this] { run_worker(); });
      std::atexit([] { shutdown(); });
    }
    cv.notify_one();
  }

  static void shutdown();

  // (mu held) load a code object into a function of the current device (nullptr on failure)
  static hipFunction_t load(const std::vector<char>& code, const char* kernel) {
    hipFunction_t fn = nullptr;
    if (code.empty()) return nullptr;
    hipModule_t mod = nullptr;
    if (hipModuleLoadData(&mod, code.data()) == hipSuccess) {
      if (hipModuleGetFunction(&fn, mod, kernel) != hipSuccess) fn = nullptr;
    } else {
      (void)hipGetLastError();
    }
    return fn;
  }
};

JitState& state() {
  static JitState* s = new JitState();  // never destroyed: modules live as long as the process
  return *s;
}

void JitState::shutdown() {
  JitState& js = state();
  {
    std::lock_guard<std::mutex> lk(js.mu);
    js.stopping = true;
    js.queue.clear();
  }
  js.cv.notify_all();
  if (js.worker.joinable()) js.worker.join();
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

hipFunction_t jit_function_for(const char* kernel, const ScanParams& p, const std::string& extra, bool async) {
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
  bool final_answer = true;
  hipFunction_t fn = jit_function(kernel, jit_spec(p) + extra, async, &final_answer);
  if (final_answer) {
    std::lock_guard<std::mutex> lk(js.mu);
    js.by_shape.emplace(std::move(key), fn);
  }
  return fn;
}

hipFunction_t jit_function(const char* kernel, const std::string& spec, bool async, bool* final_answer) {
  JitState& js = state();
  std::lock_guard<std::mutex> lk(js.mu);
  if (final_answer) *final_answer = true;
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
  // compiled in the background since the last query of this shape: load it now
  const std::string ck = std::string(kernel) + ":" + hex;  // the code object serves every device
  auto rd = js.ready.find(ck);
  if (rd != js.ready.end()) {
    hipFunction_t fn = JitState::load(rd->second, kernel);
    js.fns[key] = fn;
    return fn;
  }
  if (js.pending.count(ck)) {
    if (final_answer) *final_answer = false;
    return nullptr;  // still compiling: the generic kernel runs this query
  }
  std::vector<char> code;
  const std::string path = cache_dir() + "/" + hex + ".hsaco";
  if (async) {
    // the disk read, the compile on a miss and the module load (~1 ms even for a cached code
    // object) all run on the worker: this query runs the generic kernel
    js.enqueue(JitState::Job{ck, src, path, key, kernel, dev});
    if (final_answer) *final_answer = false;
    return nullptr;
  }
  if (!read_file(path, code)) {
    if (!js.rtc_ok()) {
      code.clear();
    } else if (js.compile(src, code)) {
      mkdirs(cache_dir());
      write_file(path, code);
    } else {
      code.clear();
    }
  }
  hipFunction_t fn = JitState::load(code, kernel);
  js.fns[key] = fn;
  return fn;
}

bool jit_wait(double timeout_ms, int64_t* compiled, int64_t* failed) {
  JitState& js = state();
  std::unique_lock<std::mutex> lk(js.mu);
  bool idle = true;
  if (timeout_ms < 0) {
    js.cv_idle.wait(lk, [&] { return js.pending.empty(); });
  } else {
    idle = js.cv_idle.wait_for(lk, std::chrono::duration<double, std::milli>(timeout_ms),
                               [&] { return js.pending.empty(); });
  }
  if (compiled) *compiled = js.compiled;
  if (failed) *failed = js.failed;
  return idle;
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
  if (js.rtc_ok() && js.compile(std::string(spec) + "#include \"jit_kernels.h\"\n", code)) return 0;
  return js.rtc && js.rtc->ok ? 2 : 1;
}
