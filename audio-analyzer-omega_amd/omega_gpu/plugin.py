"""AnalyzerPlugin drop-in (omega4/plugins/base.py:160-186).

The plugin manager takes the first ``Plugin`` subclass *defined in* the loaded file
(``_find_plugin_class``, manager.py:311-328, checks ``obj.__module__ == module.__name__``), so a
re-export is never discovered: the drop-in is ``audio-analyzer-omega_amd/plugins/omega_gpu_analyzer.py``,
which defines its own subclass of ``OmegaGPUAnalyzer``. ``PluginManager.load_plugin``
(manager.py:120-177) instantiates it with no arguments and calls ``process(audio_data, **kw)``.
When omega4 is importable the class derives from its real ``AnalyzerPlugin``; otherwise from a
local mirror of the same interface (for standalone use and the tests).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Dict, List

import numpy as np

try:  # the reference's own ABC when running inside OMEGA-4
    from omega4.plugins.base import AnalyzerPlugin, PluginMetadata, PluginType  # type: ignore
except Exception:  # pragma: no cover - standalone mirror of plugins/base.py:13-60, :160-186
    class PluginType(Enum):
        PANEL = "panel"
        ANALYZER = "analyzer"
        EFFECT = "effect"
        INPUT = "input"
        OUTPUT = "output"

    @dataclass
    class PluginMetadata:
        name: str
        version: str
        author: str
        description: str
        plugin_type: PluginType
        dependencies: List[str] = field(default_factory=list)
        config_schema: Dict = None

    class AnalyzerPlugin:
        def __init__(self):
            self._enabled = True
            self._config = {}
            self._metadata = None
            self._sample_rate = 48000

        def get_metadata(self):
            raise NotImplementedError

        def initialize(self, config: Dict = None) -> bool:
            self._metadata = self.get_metadata()
            if config:
                self._config = config
            return True

        def shutdown(self):
            pass

        def enable(self):
            self._enabled = True

        def disable(self):
            self._enabled = False

        def is_enabled(self) -> bool:
            return self._enabled

        def get_config(self) -> Dict:
            return self._config.copy()

        def set_config(self, config: Dict):
            self._config.update(config)
            self.on_config_change()

        def on_config_change(self):
            pass

        def set_sample_rate(self, sample_rate: int):
            self._sample_rate = sample_rate

        def reset(self):
            pass

import logging

from .bands import PrecomputedFrequencyMapper
from .multi_resolution_fft import MultiResolutionFFT
from .professional_meters import ProfessionalMetering

logger = logging.getLogger(__name__)


class OmegaGPUAnalyzer(AnalyzerPlugin):
    """Multi-resolution spectrum + band values + K-weighted LUFS + true peak on the MI355X.

    process(audio_data, target_bins=512, num_bars=512) ->
        {'spectrum': f32[T] combined multi-resolution spectrum (multi_resolution_fft.py:335-408),
         'bands': f32[num_bars] mel-bar means of that spectrum with the app's 2048-point base table,
                  truncated at the spectrum's end as the app's loop is (freq_mapper.py:165-196,
                  omega4_main.py:1011-1013),
         'lufs': {'momentary', 'short_term', 'integrated', 'range', 'true_peak'} (professional_meters.py:231-281),
         'true_peak': float, 'frequencies': f64[T]}

    Errors are logged and the previous result (or {}) returned -- the reference's never-raise
    convention for the analysis path. The GPU is touched on the first process()
    call, not at construction (the plugin manager instantiates and initialises plugins up front).
    """

    APP_FFT_BASE = 2048  # omega4_main.py:171: the bar table is built for a 2048-point FFT

    def __init__(self):
        super().__init__()
        self._mrfft = None
        self._meter = None
        self._mapper = None
        self._last: Dict[str, Any] = {}

    def get_metadata(self) -> PluginMetadata:
        return PluginMetadata(name="omega_gpu_analyzer", version="0.2", author="omega-mi355x",
                              description="MI355X multi-resolution FFT, band values, LUFS and true peak",
                              plugin_type=PluginType.ANALYZER)

    def _ensure(self, num_bars: int):
        if self._mrfft is None:
            self._mrfft = MultiResolutionFFT(self._sample_rate)
            self._meter = ProfessionalMetering(self._sample_rate)
        if self._mapper is None or self._mapper.num_bars != num_bars:
            self._mapper = PrecomputedFrequencyMapper(self._sample_rate, self.APP_FFT_BASE, num_bars)

    def set_sample_rate(self, sample_rate: int):
        super().set_sample_rate(sample_rate)
        self._mrfft = self._meter = self._mapper = None

    def process(self, audio_data: np.ndarray, **kwargs) -> Dict[str, Any]:
        try:
            t = int(kwargs.get("target_bins", 512))
            nb = int(kwargs.get("num_bars", 512))
            self._ensure(nb)
            res = self._mrfft.process_audio_chunk(audio_data)
            spec, freqs = self._mrfft.combine_results_optimized(res, t)
            lufs = dict(self._meter.calculate_lufs(audio_data))
            bands = self._mapper.map_spectrum_to_bars(spec, apply_compensation=False)
            self._last = {"spectrum": spec, "bands": bands, "lufs": lufs, "true_peak": lufs["true_peak"],
                          "frequencies": freqs}
        except Exception as e:  # the reference logs and keeps the previous values
            logger.error("OmegaGPUAnalyzer.process failed: %s", e)
        return self._last

    def reset(self):
        if self._mrfft is not None:
            self._mrfft.reset_all_buffers()
            self._meter.reset()
        self._last = {}
