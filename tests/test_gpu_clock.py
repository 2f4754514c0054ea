"""rsh_debug_k1_clock (include/rsync_hip_debug.h): the clock the chip holds under the Generator's K1, from a stamped
diagnostic instantiation of the production body (per-wave s_memtime / s_memrealtime).  bench.py reports it as
roofline.k1_clock_ghz; here it must be a plausible MI355X clock (<= 2.4 GHz peak) and reject shapes the diagnostic
kernel does not run (partial waves, B not a multiple of 128)."""
import ctypes

import pytest

import rsync_hip as R

pytestmark = pytest.mark.gpu


def test_k1_clock_plausible():
    R.build()
    with R.Context(0) as ctx:
        n, B = 1 << 30, 131072
        d = ctx.alloc(n)
        assert R.lib().rsh_fill_splitmix_device(ctx.handle, d.ptr, n, 0xC10C, 0) == 0
        ghz = ctypes.c_double()
        assert R.lib().rsh_debug_k1_clock(ctx.handle, d.ptr, n, B, 2, ctypes.byref(ghz)) == 0
        assert 0.5 < ghz.value <= 2.5, ghz.value
        assert R.lib().rsh_debug_k1_clock(ctx.handle, d.ptr, n - B, B, 1, ctypes.byref(ghz)) == R.RSH_E_INVAL
        assert R.lib().rsh_debug_k1_clock(ctx.handle, d.ptr, 64 * 1000, 1000, 1, ctypes.byref(ghz)) == R.RSH_E_INVAL
        d.free()
