"""roctx tracing hooks (csrc/runtime/trace.cpp; SURVEY §5 tracing): the roctx library is
dlopen'ed lazily only when tracing is switched on (MIINT_ROCTX=1 or enable_tracing), ranges
and marks are no-ops otherwise. CPU only: the ROCm roctx library loads without a GPU."""
from __future__ import annotations


def test_tracing_toggle_and_marks(native):
    native.enable_tracing(False)
    assert not native.tracing_enabled()
    native.trace_mark("miint.test.off")          # no-op while disabled
    native.enable_tracing(True)
    on = native.tracing_enabled()                # True iff a roctx library was found
    native.trace_mark("miint.test.on")
    native.enable_tracing(False)
    assert not native.tracing_enabled()
    assert on in (True, False)
