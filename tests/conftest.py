import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


import pytest  # noqa: E402


class _OptionPatch:
    """monkeypatch-like setter of the library options (include/gibbs_capi.h
    gs_option_set; the library reads no environment variables): every option
    set through it is restored when the test ends."""

    def __init__(self):
        self._saved = {}

    def setenv(self, name, value):
        from gibbssampler_amd import _capi
        if name not in self._saved:
            self._saved[name] = _capi.get_option(name)
        _capi.set_option(name, value)

    def delenv(self, name, raising=False):
        self.setenv(name, None)

    def undo(self):
        from gibbssampler_amd import _capi
        for k, v in self._saved.items():
            _capi.set_option(k, v)
        self._saved.clear()


@pytest.fixture
def gsopt():
    p = _OptionPatch()
    yield p
    p.undo()
