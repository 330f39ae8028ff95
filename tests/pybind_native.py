"""Load the built pybind11 module (fhe-fed_amd/pybind/SHELFI_FHE*.so, INTEGRATION.md
Option B) beside the ctypes package of the same name: the extension is created from its
file without entering sys.modules, so both stay importable in one test process."""
import glob
import importlib.machinery
import importlib.util
import os
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATH = os.path.join(ROOT, "fhe-fed_amd", "pybind", "SHELFI_FHE" + sysconfig.get_config_var("EXT_SUFFIX"))

_mod = None


def load():
    global _mod
    if _mod is None:
        if not os.path.exists(PATH):
            raise ImportError("%s is not built (make -C fhe-fed_amd/csrc; found %s)"
                              % (PATH, glob.glob(os.path.join(os.path.dirname(PATH), "*.so"))))
        loader = importlib.machinery.ExtensionFileLoader("SHELFI_FHE", PATH)
        spec = importlib.util.spec_from_file_location("SHELFI_FHE", PATH, loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _mod = mod
    return _mod
