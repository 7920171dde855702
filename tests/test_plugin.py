"""The AnalyzerPlugin drop-in: the plugin file is discoverable by the reference's
plugin manager, constructs and initialises without a GPU, and (on the GPU) process() returns the
§8(b) keys with the oracle's values."""
import importlib.util
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, load_golden, normwise

PKG = os.path.join(REPO, "audio-analyzer-omega_amd")
DROPIN = os.path.join(PKG, "plugins", "omega_gpu_analyzer.py")
REF = "/root/reference"


def _load_as_plugin_manager_does(path, name="omega4_plugins.analyzers.omega_gpu_analyzer"):
    """manager.py:131-144: spec_from_file_location under the generated module name, exec_module."""
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def _find_plugin_class(module, plugin_base, base_classes):
    """The predicate of manager.py:311-328, restated: the first public Plugin subclass that is not a
    base class and is defined in the module itself."""
    for name in dir(module):
        obj = getattr(module, name)
        if (isinstance(obj, type) and issubclass(obj, plugin_base) and obj not in base_classes
                and not name.startswith("_") and getattr(obj, "__module__", None) == module.__name__):
            return obj
    return None


def test_dropin_is_discovered_and_initialises_without_gpu():
    from omega_gpu import plugin as P
    mod = _load_as_plugin_manager_does(DROPIN)
    cls = _find_plugin_class(mod, P.AnalyzerPlugin, {P.AnalyzerPlugin})
    assert cls is not None and cls.__name__ == "OmegaGPUAnalyzer"
    assert issubclass(cls, P.OmegaGPUAnalyzer)
    # a re-export (what round 1 documented) is NOT discovered
    reexp = type(sys)("omega4_plugins.reexport")
    reexp.OmegaGPUAnalyzer = P.OmegaGPUAnalyzer
    assert _find_plugin_class(reexp, P.AnalyzerPlugin, {P.AnalyzerPlugin}) is None
    inst = cls()                              # manager.py:147: no-argument constructor
    assert inst.initialize({}) is True        # :153
    md = inst.get_metadata()
    assert md.name == "omega_gpu_analyzer" and md.plugin_type.value == "analyzer"
    inst.set_sample_rate(44100)
    inst.reset()


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference is only present in the build container")
def test_reference_plugin_manager_loads_dropin(tmp_path):
    """The reference's own PluginManager.load_plugin on the drop-in file (in a subprocess with the
    reference on sys.path, so omega_gpu.plugin derives from the real AnalyzerPlugin)."""
    d = tmp_path / "plugins"
    d.mkdir()
    (d / "omega_gpu_analyzer.py").write_text(open(DROPIN).read())
    code = (
        "import sys\n"
        "from omega4.plugins.manager import PluginManager\n"
        "from omega4.plugins.base import AnalyzerPlugin\n"
        f"pm = PluginManager([{str(d)!r}])\n"
        f"p = pm.load_plugin({str(d / 'omega_gpu_analyzer.py')!r})\n"
        "assert p is not None, 'not loaded'\n"
        "assert isinstance(p, AnalyzerPlugin)\n"
        "assert pm.get_plugin('omega_gpu_analyzer') is p\n"
        "print('loaded', type(p).__module__)\n")
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([REF, PKG]), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "loaded omega4_plugins" in r.stdout


@pytest.mark.gpu
def test_plugin_process_matches_oracle():
    """process() on golden frames (the reference's default resolutions): spectrum vs the oracle's
    combine(512), bands vs the oracle's mel bars of that spectrum (2048-point base table, truncated
    at the spectrum's end), LUFS aggregates and true peak vs the oracle's meter state."""
    from oracle import omega_ref as R
    from omega_gpu import plugin as P
    g = load_golden("mrfft")
    frames = [np.asarray(g[k], np.float32) for k in ("triad_4096/x", "comp_4096/x")] * 2
    a = P.OmegaGPUAnalyzer()
    assert a.initialize({})
    st = R.MeterState(48000)
    table = R.mel_band_table(48000, 2048, 512)
    for fr in frames:
        out = a.process(fr, target_bins=512)
        assert set(out) >= {"spectrum", "bands", "lufs", "true_peak"}
        _, comb, li, tp = R.full_frame(fr, configs=R.DEFAULT_CONFIGS, target_bins=512)
        assert normwise(out["spectrum"], comb) < 1e-4
        bars = R.map_spectrum_to_bars(out["spectrum"], table, None, 512, apply_compensation=False)
        np.testing.assert_allclose(out["bands"], bars, rtol=2e-6, atol=1e-9)
        st.update(fr, li, tp)
        for k in ("momentary", "short_term", "integrated", "range"):
            assert abs(out["lufs"][k] - st.current[k]) < 0.1, k
        assert abs(out["true_peak"] - st.current["true_peak"]) < 0.01
    last = a.process(fr)
    assert a.process(None) is last  # never raises: logs and keeps the previous result
