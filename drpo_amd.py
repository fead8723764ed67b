"""Import alias for the package directory ``distributional-reachability-policy-optimization_amd/``
(the repository layout requires that hyphenated name, which is not a valid module
name): ``import drpo_amd`` loads it as a regular package."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'distributional-reachability-policy-optimization_amd')
_spec = importlib.util.spec_from_file_location(__name__, os.path.join(_DIR, '__init__.py'),
                                               submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
