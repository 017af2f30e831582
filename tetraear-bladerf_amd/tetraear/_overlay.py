"""The reference package behind this build (INTEGRATION.md option A: the drop-in overlay).

This build provides the receive hot path only: ``tetraear.signal.processor`` / ``.scanner`` and
``tetraear.core.decoder`` / ``.protocol`` (plus its own modules).  Put its package root ahead of the
reference's on ``sys.path`` -- or name the reference's root in ``TETRAEAR_REFERENCE_ROOT`` -- and
each package of the build (``tetraear``, ``tetraear.signal``, ``tetraear.core``) extends its
``__path__`` with the reference's same directory.  The reference's unchanged callers then get:

* the build's modules wherever it has one (they shadow the reference's files);
* every other module from the reference, unchanged: ``signal.capture``, ``core.crypto``,
  ``core.mcc_mnc``, ``core.validator``, ``core.location``, ``audio``, ``ui``, ``tools``
  (/root/reference/tetraear/ui/modern.py:193-201 imports all of them);
* the non-hot-path members of the four shadowed modules, from the reference's own file loaded
  under a private module name (``reference_module``): ``FrequencyScanner`` (scanner.py:292-554,
  given the build's GPU detector), ``TetraDecoder``'s key setup / decryption / formatting
  (decoder.py:36-138, 576-834, 1121-1200) and ``TetraProtocolParser``'s upper MAC
  (protocol.py:597-1300: call metadata, SDS, LIP, GSM 7-bit).

The hot path never delegates: ``process``, ``decode``, ``parse_burst``, ``_check_crc``,
``_calculate_crc16`` and ``parse_mac_pdu`` are the build's methods with or without the overlay.
Without a reference on the path nothing here is active: the build runs alone and the upper-MAC
members raise ``ReferenceUnavailable`` naming what is missing.
"""
import importlib.util
import inspect
import os
import sys
import threading

_HERE = os.path.realpath(os.path.dirname(os.path.abspath(__file__)))   # this build's tetraear/
_lock = threading.Lock()
_loaded = {}


class ReferenceUnavailable(ImportError):
    """A member outside the hot path was asked for and no reference package is on the path."""


_scan = (None, ())


# files only a copy of THIS build has: such a package is never taken for the reference (a second
# checkout or an installed wheel beside the source tree would otherwise load its own parser as "the
# reference's" and recurse through this module again)
_BUILD_MARKERS = ("_overlay.py", "_hip.py")


def _is_build_copy(d):
    return any(os.path.isfile(os.path.join(d, m)) for m in _BUILD_MARKERS)


def reference_packages():
    """The reference's ``tetraear/`` directories: ``$TETRAEAR_REFERENCE_ROOT/tetraear`` first, then
    (unless ``TETRAEAR_OVERLAY=0``) every other ``tetraear`` package on ``sys.path``, in path order --
    never this build's own nor another copy of it.  Cached until sys.path or the variables change
    (upper_mac asks once per frame)."""
    global _scan
    scan = os.environ.get("TETRAEAR_OVERLAY", "1") != "0"
    key = (os.environ.get("TETRAEAR_REFERENCE_ROOT"), scan, tuple(p for p in sys.path if isinstance(p, str)))
    if _scan[0] == key:
        return list(_scan[1])
    roots = []
    env = os.environ.get("TETRAEAR_REFERENCE_ROOT")
    if env:
        roots.append(env)
    if scan:
        roots += [p or os.getcwd() for p in sys.path if isinstance(p, str)]
    out = []
    for r in roots:
        d = os.path.realpath(os.path.join(r, "tetraear"))
        if d != _HERE and d not in out and os.path.isfile(os.path.join(d, "__init__.py")) and not _is_build_copy(d):
            out.append(d)
    _scan = (key, tuple(out))
    return out


def active():
    return bool(reference_packages())


def extend(path, name):
    """``__path__`` of the build's package ``name`` followed by the reference's directories for it."""
    rel = name.split(".")[1:]
    out = list(path)
    seen = {os.path.realpath(p) for p in out}
    for pkg in reference_packages():
        d = os.path.join(pkg, *rel)
        if os.path.isdir(d) and os.path.realpath(d) not in seen:
            out.append(d)
            seen.add(os.path.realpath(d))
    return out


def reference_module(rel, patch=None):
    """The reference's own module ``tetraear/<rel>.py`` that this build shadows (rel like
    "core/protocol"), executed once from the reference's file under the private name
    ``_tetraear_reference.<rel>``.  Its absolute imports resolve through the overlay (the build's
    hot-path modules, the reference's others).  ``patch`` (name -> object) replaces module globals
    after loading -- the build's enums / dataclasses, so values cross between the two modules
    unchanged.  Raises ReferenceUnavailable when no reference is on the path."""
    with _lock:
        if rel in _loaded:
            return _loaded[rel]
        for pkg in reference_packages():
            f = os.path.join(pkg, *rel.split("/")) + ".py"
            if os.path.isfile(f):
                break
        else:
            raise ReferenceUnavailable(
                f"tetraear/{rel}.py beyond the hot path is the reference's: put the reference's package root on "
                f"sys.path after this build's, or set TETRAEAR_REFERENCE_ROOT (INTEGRATION.md option A)")
        name = "_tetraear_reference." + rel.replace("/", ".")
        spec = importlib.util.spec_from_file_location(name, f)
        mod = importlib.util.module_from_spec(spec)
        sys.modules[name] = mod   # dataclasses resolve their module through sys.modules
        try:
            spec.loader.exec_module(mod)
        except BaseException:
            del sys.modules[name]
            raise
        for k, v in (patch or {}).items():
            setattr(mod, k, v)
        _loaded[rel] = mod
        return mod


def bind(obj, cls, name):
    """Attribute ``name`` of the reference class ``cls`` as seen from ``obj`` (a build instance):
    functions become methods bound to ``obj``, other class attributes are returned as they are."""
    raw = inspect.getattr_static(cls, name)
    if isinstance(raw, staticmethod):
        return raw.__func__
    if isinstance(raw, classmethod):
        return raw.__get__(None, cls)
    if isinstance(raw, property) or (inspect.isfunction(raw)):
        return raw.__get__(obj, type(obj))
    return raw
