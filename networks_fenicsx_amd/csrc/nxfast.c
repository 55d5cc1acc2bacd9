/* The per-step host calls of the direct step (nx_assemble, nx_solve) without ctypes: a
 * CPython extension holding the two C-ABI entry points of the already loaded libnxhip.so
 * (their addresses come from ctypes at import, so this module links nothing). ctypes costs
 * ~1 us per call with its argument conversion and out-parameters; this path ~0.1 us. It is
 * host plumbing only: the same C entry points run, and _lib.Handle falls back to ctypes
 * when this module is missing. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>
#include <stdint.h>

typedef int (*assemble_fn)(void*, int32_t, int32_t);
typedef int (*solve_fn)(void*, double, int32_t, int32_t, int32_t*, double*, int32_t*);

static assemble_fn g_assemble = NULL;
static solve_fn g_solve = NULL;

/* bind(assemble_addr, solve_addr) */
static PyObject* nxf_bind(PyObject* self, PyObject* args) {
  unsigned long long a = 0, s = 0;
  (void)self;
  if (!PyArg_ParseTuple(args, "KK", &a, &s)) return NULL;
  g_assemble = (assemble_fn)(uintptr_t)a;
  g_solve = (solve_fn)(uintptr_t)s;
  Py_RETURN_NONE;
}

/* assemble(handle, lhs, rhs) -> rc */
static PyObject* nxf_assemble(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 3 || !g_assemble) {
    PyErr_SetString(PyExc_RuntimeError, "nxfast.assemble(handle, lhs, rhs) after bind()");
    return NULL;
  }
  void* h = PyLong_AsVoidPtr(args[0]);
  const long lhs = PyLong_AsLong(args[1]), rhs = PyLong_AsLong(args[2]);
  if (PyErr_Occurred()) return NULL;
  return PyLong_FromLong(g_assemble(h, (int32_t)lhs, (int32_t)rhs));
}

/* solve(handle, rtol, maxit, check_every) -> (rc, it, relres, converged) */
static PyObject* nxf_solve(PyObject* self, PyObject* const* args, Py_ssize_t n) {
  (void)self;
  if (n != 4 || !g_solve) {
    PyErr_SetString(PyExc_RuntimeError, "nxfast.solve(handle, rtol, maxit, every) after bind()");
    return NULL;
  }
  void* h = PyLong_AsVoidPtr(args[0]);
  const double rtol = PyFloat_AsDouble(args[1]);
  const long maxit = PyLong_AsLong(args[2]), every = PyLong_AsLong(args[3]);
  if (PyErr_Occurred()) return NULL;
  int32_t it = 0, conv = 0;
  double rr = 0.0;
  int rc;
  /* (the solve spins on the published state: let other Python threads run meanwhile) */
  Py_BEGIN_ALLOW_THREADS
  rc = g_solve(h, rtol, (int32_t)maxit, (int32_t)every, &it, &rr, &conv);
  Py_END_ALLOW_THREADS
  return Py_BuildValue("(iidO)", rc, (int)it, rr, conv ? Py_True : Py_False);
}

static PyMethodDef nxf_methods[] = {
    {"bind", nxf_bind, METH_VARARGS, "bind(assemble_addr, solve_addr)"},
    {"assemble", (PyCFunction)(void (*)(void))nxf_assemble, METH_FASTCALL,
     "assemble(handle, lhs, rhs) -> rc"},
    {"solve", (PyCFunction)(void (*)(void))nxf_solve, METH_FASTCALL,
     "solve(handle, rtol, maxit, check_every) -> (rc, it, relres, converged)"},
    {NULL, NULL, 0, NULL}};

static struct PyModuleDef nxf_module = {PyModuleDef_HEAD_INIT, "_nxfast", NULL, -1, nxf_methods,
                                        NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__nxfast(void) { return PyModule_Create(&nxf_module); }
