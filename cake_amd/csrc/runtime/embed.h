// Embedded Python compute runtime for the native entry points.
//
// The native binaries (cake-cli) and the C ABI (cake_start_worker) own the
// process: they parse and validate the flags, resolve the topology, and the
// worker's TCP server is the native WorkerServer; the tensor compute
// (PyTorch-ROCm + the gfx950 HIP kernels) runs in an interpreter embedded in
// the SAME process — no child process, no exec.
#pragma once

#include <map>
#include <string>

namespace cake {

struct PyArg {
  enum Kind { kStr, kInt, kFloat, kBool, kNone } kind = kNone;
  std::string value;
};

using PyArgs = std::map<std::string, PyArg>;  // argparse dest -> typed value

// Run cake_amd.cli.run_parsed(options) in the embedded interpreter (initialising
// it if this process has none; from a thread of a process that already runs
// Python it takes the GIL of that interpreter).  Returns the run's exit code
// (1 + a printed traceback on an uncaught exception).
int run_embedded(const PyArgs& options);

// Call `module.function(arg)` in the embedded interpreter (initialised on first use,
// GIL taken for the call) with one str argument; returns the str result.  Throws
// std::runtime_error (with the Python traceback printed) on failure.  The native text
// path uses it for the tokenizer only (cake_amd/native_bridge.py).
std::string call_python(const std::string& module, const std::string& function,
                        const std::string& arg);

// Directory that contains the cake_amd package (derived from the location of
// the code object this function lives in), for sys.path.
std::string package_root();

}  // namespace cake
