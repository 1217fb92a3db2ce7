"""Import the REAL reference package (`fastgps`, read-only at /root/reference) in this container.

TEST INFRASTRUCTURE ONLY: used by tests/golden/make_golden.py (golden-vector generation) and
by CPU tests that cross-check the oracle against the live reference when /root/reference exists.
Never imported by the product package; /root/reference does not exist on the GPU box.

Two shims (probed there):
  1. Syntax: abstract_gp.py:228,248,249,258,259,272 use PEP-646 `x[...,*masks]` (Python >= 3.11).
     The source is read AS TEXT at import time and those subscripts are rewritten in memory to the
     equivalent tuple form `x[(...,*masks)]`; nothing is written anywhere (no bytecode, no files).
  2. `qmcpy` is absent: oracle/refshim/qmcpy is a stand-in restating its published algorithms.
"""
import importlib.abc
import importlib.machinery
import importlib.util
import os
import re
import sys

REFERENCE_ROOT = os.environ.get("FGP_REFERENCE_ROOT", "/root/reference")
_PKG = "fastgps"
_HERE = os.path.dirname(os.path.abspath(__file__))

_REWRITES = [
    (re.compile(r"\[\.\.\.,\*masks,:\]"), "[(...,*masks,slice(None))]"),
    (re.compile(r"\[\.\.\.,\*masks,0\]"), "[(...,*masks,0)]"),
    (re.compile(r"\[\.\.\.,\*masks\]"), "[(...,*masks)]"),
]


def reference_available():
    return os.path.isfile(os.path.join(REFERENCE_ROOT, _PKG, "__init__.py"))


class _RefLoader(importlib.abc.Loader):
    def __init__(self, path):
        self.path = path

    def create_module(self, spec):
        return None

    def exec_module(self, module):
        with open(self.path, "r") as f:
            src = f.read()
        for pat, rep in _REWRITES:
            src = pat.sub(rep, src)
        code = compile(src, self.path, "exec", dont_inherit=True)
        exec(code, module.__dict__)


class _RefFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path, target=None):
        if fullname != _PKG and not fullname.startswith(_PKG + "."):
            return None
        pkgdir = os.path.join(REFERENCE_ROOT, _PKG)
        if fullname == _PKG:
            fpath = os.path.join(pkgdir, "__init__.py")
            spec = importlib.machinery.ModuleSpec(fullname, _RefLoader(fpath), origin=fpath, is_package=True)
            spec.submodule_search_locations = [pkgdir]
            spec.has_location = True
            return spec
        sub = fullname[len(_PKG) + 1:]
        fpath = os.path.join(pkgdir, *sub.split(".")) + ".py"
        if not os.path.isfile(fpath):
            return None
        spec = importlib.machinery.ModuleSpec(fullname, _RefLoader(fpath), origin=fpath)
        spec.has_location = True
        return spec


def import_reference():
    """Return the reference `fastgps` module (with the qmcpy stand-in on sys.path)."""
    if not reference_available():
        raise ImportError("reference not present at %s" % REFERENCE_ROOT)
    sys.dont_write_bytecode = True
    if _HERE not in sys.path:
        sys.path.insert(0, _HERE)
    if not any(isinstance(f, _RefFinder) for f in sys.meta_path):
        sys.meta_path.insert(0, _RefFinder())
    import fastgps  # noqa: E402  (resolved by _RefFinder)
    import qmcpy  # noqa: E402  (the stand-in)
    assert qmcpy.__version__.startswith("standin"), "a real qmcpy shadowed the stand-in"
    return fastgps
