"""AnalyzerPlugin drop-in (omega4/plugins/base.py:160-186).

Drop this module (or a one-line file importing ``OmegaGPUAnalyzer``) into an OMEGA-4 plugin
directory: ``PluginManager.load_plugin`` (manager.py:120-177) instantiates the first ``Plugin``
subclass defined in the module with no arguments and calls ``process(audio_data, **kw)``.
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

from .multi_resolution_fft import MultiResolutionFFT
from .professional_meters import ProfessionalMetering


class OmegaGPUAnalyzer(AnalyzerPlugin):
    """Multi-resolution spectrum + K-weighted LUFS + true peak on the MI355X.

    process(audio_data, target_bins=512) -> {'spectrum', 'frequencies', 'lufs': {...}, 'true_peak'}
    """

    def __init__(self):
        super().__init__()
        self._mrfft = None
        self._meter = None

    def get_metadata(self) -> PluginMetadata:
        return PluginMetadata(name="omega_gpu_analyzer", version="0.1", author="omega-mi355x",
                              description="MI355X multi-resolution FFT, LUFS and true peak",
                              plugin_type=PluginType.ANALYZER)

    def _ensure(self):
        if self._mrfft is None:
            self._mrfft = MultiResolutionFFT(self._sample_rate)
            self._meter = ProfessionalMetering(self._sample_rate)

    def set_sample_rate(self, sample_rate: int):
        super().set_sample_rate(sample_rate)
        self._mrfft = self._meter = None

    def process(self, audio_data: np.ndarray, **kwargs) -> Dict[str, Any]:
        self._ensure()
        t = int(kwargs.get("target_bins", 512))
        res = self._mrfft.process_audio_chunk(audio_data)
        spec, freqs = self._mrfft.combine_results_optimized(res, t)
        lufs = dict(self._meter.calculate_lufs(audio_data))
        return {"spectrum": spec, "frequencies": freqs, "lufs": lufs, "true_peak": lufs["true_peak"]}

    def reset(self):
        if self._mrfft is not None:
            self._mrfft.reset_all_buffers()
            self._meter.reset()
