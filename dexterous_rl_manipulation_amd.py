"""Import shim: the package directory is named `dexterous-rl-manipulation_amd`
(not a valid Python identifier).  `import dexterous_rl_manipulation_amd` loads
that directory as the package and replaces this module with it."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dexterous-rl-manipulation_amd")
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_DIR, "__init__.py"),
                                               submodule_search_locations=[_DIR])
_pkg = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _pkg
_spec.loader.exec_module(_pkg)
