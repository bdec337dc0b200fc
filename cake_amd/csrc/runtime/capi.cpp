// Embeddable worker entry point (C ABI).
//
// Counterpart of the reference's uniffi export
// `start_worker(name, model_path, topology_path, model_type)`
// (cake-ios/src/lib.rs:6-87), which runs a worker on 0.0.0.0:10128 with
// default args.  Here the worker runtime lives in the cake_amd package, so the
// C entry point spawns it as a child process (posix_spawnp, never exec in the
// calling process — it may already own a GPU context) and returns its exit
// status when it stops.
#include <spawn.h>
#include <sys/wait.h>

#include <string>
#include <vector>

extern char** environ;

extern "C" __attribute__((visibility("default"))) int cake_start_worker(
    const char* name, const char* model_path, const char* topology_path, const char* model_type,
    const char* address) {
  std::vector<std::string> args = {"python3", "-m", "cake_amd.cli", "--mode", "worker",
                                   "--name", name ? name : "worker",
                                   "--model", model_path ? model_path : ".",
                                   "--topology", topology_path ? topology_path : "topology.yml",
                                   "--address", address && *address ? address : "0.0.0.0:10128"};
  const std::string mt = model_type ? model_type : "text";
  args.push_back("--model-type");
  args.push_back(mt == "image" ? "image-model" : "text-model");
  std::vector<char*> argv;
  for (auto& a : args) argv.push_back(&a[0]);
  argv.push_back(nullptr);
  pid_t pid;
  if (posix_spawnp(&pid, "python3", nullptr, nullptr, argv.data(), environ) != 0) return -1;
  int status = 0;
  if (waitpid(pid, &status, 0) < 0) return -1;
  return WIFEXITED(status) ? WEXITSTATUS(status) : -1;
}
