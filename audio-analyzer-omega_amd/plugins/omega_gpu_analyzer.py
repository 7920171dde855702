"""OMEGA-4 plugin drop-in: copy this file into a plugin directory (e.g. omega4/plugins/analyzers/).

PluginManager.load_plugin (omega4/plugins/manager.py:120-177) executes the file as its own module and
instantiates the first Plugin subclass *defined here* (_find_plugin_class, manager.py:311-328: the
class's __module__ must be the loaded module's name), with no arguments. The implementation lives in
omega_gpu.plugin; the class below only gives it this module as its home. omega_gpu is found on
sys.path (INTEGRATION.md §0 exports it) or under $OMEGA_GPU_HOME.
"""
import os
import sys

try:
    import omega_gpu  # noqa: F401
except ImportError:  # pragma: no cover - a copy outside the repo with OMEGA_GPU_HOME set
    _home = os.environ.get("OMEGA_GPU_HOME", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, _home)
    import omega_gpu  # noqa: F401

from omega_gpu.plugin import OmegaGPUAnalyzer as _OmegaGPUAnalyzerImpl


class OmegaGPUAnalyzer(_OmegaGPUAnalyzerImpl):
    """The MI355X analyzer (omega_gpu.plugin.OmegaGPUAnalyzer), defined in this module for discovery."""
