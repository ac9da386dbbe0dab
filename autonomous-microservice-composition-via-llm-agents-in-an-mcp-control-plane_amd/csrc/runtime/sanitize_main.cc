// Host sanitizer harness for the native runtime.
//
// The runtime (runtime.cpp) is normally a pybind11 extension loaded by an
// uninstrumented python, where AddressSanitizer would need its runtime
// preloaded.  Instead this executable IS the instrumented process: it compiles
// runtime.cpp in with -fsanitize=address,undefined, registers the module as a
// built-in (_runtime_san) and embeds the interpreter to run a fuzz script
// (sanitize_fuzz.py) against it.  Any heap overflow, use-after-free or UB in
// the allocator, the step packer, the topological sort, the grammar decoder or the
// feature-hashing embedder
// aborts the run.
//
// Build + run: tests/test_runtime_sanitize_cpu.py (host only; GPU sanitizers
// are not available on the MI355X pool).
#define MODULE_NAME _runtime_san
#include "runtime.cpp"
#include "grammar.cpp"
#include "embed.cpp"

#include <pybind11/embed.h>

#include <cstdio>

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s fuzz_script.py [args...]\n", argv[0]);
    return 2;
  }
  if (PyImport_AppendInittab("_runtime_san", PyInit__runtime_san) == -1) return 3;
  py::scoped_interpreter guard{};
  try {
    py::list pyargv;
    for (int i = 1; i < argc; ++i) pyargv.append(argv[i]);
    py::module_::import("sys").attr("argv") = pyargv;
    py::eval_file(argv[1]);
  } catch (const py::error_already_set& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
