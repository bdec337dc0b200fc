// See embed.h.
#include "embed.h"

#include <Python.h>
#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace cake {

std::string package_root() {
  // <root>/cake_amd/lib/<this .so or executable>  ->  <root>
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(&package_root), &info) && info.dli_fname) {
    char buf[4096];
    const char* p = realpath(info.dli_fname, buf);
    std::string s = p ? p : info.dli_fname;
    for (int i = 0; i < 3; ++i) {
      const auto cut = s.find_last_of('/');
      if (cut == std::string::npos) return ".";
      s = s.substr(0, cut);
    }
    return s.empty() ? "/" : s;
  }
  return ".";
}

static PyObject* to_py(const PyArg& a) {
  switch (a.kind) {
    case PyArg::kStr: return PyUnicode_FromString(a.value.c_str());
    case PyArg::kInt: return PyLong_FromLongLong(std::strtoll(a.value.c_str(), nullptr, 10));
    case PyArg::kFloat: return PyFloat_FromDouble(std::strtod(a.value.c_str(), nullptr));
    case PyArg::kBool: return PyBool_FromLong(a.value == "1" || a.value == "true");
    case PyArg::kNone: break;
  }
  Py_RETURN_NONE;
}

// Start the interpreter if this process has none (the GIL is released afterwards:
// every call takes it through PyGILState).
static bool ensure_interpreter() {
  if (Py_IsInitialized()) return true;
  PyConfig cfg;
  PyConfig_InitPythonConfig(&cfg);
  cfg.install_signal_handlers = 1;  // Ctrl-C -> KeyboardInterrupt, like the CLI
  cfg.parse_argv = 0;
  const PyStatus st = Py_InitializeFromConfig(&cfg);
  PyConfig_Clear(&cfg);
  if (PyStatus_Exception(st)) {
    std::fprintf(stderr, "cake: cannot start the embedded Python runtime\n");
    return false;
  }
  PyEval_SaveThread();
  return true;
}

static void add_root_to_path() {
  PyObject* sys_path = PySys_GetObject("path");  // borrowed
  PyObject* root = PyUnicode_FromString(package_root().c_str());
  if (sys_path && root && !PySequence_Contains(sys_path, root)) PyList_Insert(sys_path, 0, root);
  Py_XDECREF(root);
}

std::string call_python(const std::string& module, const std::string& function,
                        const std::string& arg) {
  if (!ensure_interpreter()) throw std::runtime_error("no Python runtime");
  const PyGILState_STATE gil = PyGILState_Ensure();
  add_root_to_path();
  PyObject* mod = PyImport_ImportModule(module.c_str());
  PyObject* fn = mod ? PyObject_GetAttrString(mod, function.c_str()) : nullptr;
  PyObject* a = PyUnicode_FromStringAndSize(arg.data(), (Py_ssize_t)arg.size());
  PyObject* res = (fn && a) ? PyObject_CallOneArg(fn, a) : nullptr;
  std::string out;
  bool ok = false;
  if (res && PyUnicode_Check(res)) {
    Py_ssize_t n = 0;
    const char* u = PyUnicode_AsUTF8AndSize(res, &n);
    if (u) {
      out.assign(u, (size_t)n);
      ok = true;
    }
  }
  if (!ok && PyErr_Occurred()) PyErr_Print();
  Py_XDECREF(res);
  Py_XDECREF(a);
  Py_XDECREF(fn);
  Py_XDECREF(mod);
  PyGILState_Release(gil);
  if (!ok) throw std::runtime_error(module + "." + function + " failed");
  return out;
}

int run_embedded(const PyArgs& options) {
  const bool owner = !Py_IsInitialized();
  if (!ensure_interpreter()) return 1;
  const PyGILState_STATE gil = PyGILState_Ensure();
  int rc = 1;
  add_root_to_path();
  PyObject* mod = PyImport_ImportModule("cake_amd.cli");
  PyObject* fn = mod ? PyObject_GetAttrString(mod, "run_parsed") : nullptr;
  PyObject* kw = PyDict_New();
  for (const auto& kv : options) {
    PyObject* v = to_py(kv.second);
    PyDict_SetItemString(kw, kv.first.c_str(), v);
    Py_DECREF(v);
  }
  PyObject* res = fn ? PyObject_CallOneArg(fn, kw) : nullptr;
  if (res) {
    rc = PyLong_Check(res) ? (int)PyLong_AsLong(res) : 0;
  } else if (PyErr_ExceptionMatches(PyExc_SystemExit)) {
    PyObject *t, *v, *tb;
    PyErr_Fetch(&t, &v, &tb);
    PyObject* code = v ? PyObject_GetAttrString(v, "code") : nullptr;
    rc = (code && PyLong_Check(code)) ? (int)PyLong_AsLong(code) : (code == Py_None ? 0 : 1);
    Py_XDECREF(code);
    Py_XDECREF(t); Py_XDECREF(v); Py_XDECREF(tb);
  } else {
    if (PyErr_ExceptionMatches(PyExc_KeyboardInterrupt)) rc = 130;
    PyErr_Print();
  }
  Py_XDECREF(res);
  Py_XDECREF(kw);
  Py_XDECREF(fn);
  Py_XDECREF(mod);
  // the interpreter is not finalised: flush Python's own stdio buffers now
  PyRun_SimpleString("import sys\nfor _s in (sys.stdout, sys.stderr):\n    try:\n"
                     "        _s.flush()\n    except Exception:\n        pass\n");
  std::fflush(stdout);
  PyGILState_Release(gil);
  // the interpreter is left alive: finalising with the GPU runtime loaded gains
  // nothing at process exit and a later cake_start_worker call may reuse it
  (void)owner;
  return rc;
}

}  // namespace cake
