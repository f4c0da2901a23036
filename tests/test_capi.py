"""CPU: the C-ABI library loads, exports every symbol include/rsort.h declares, and validates
options before touching the GPU (errors mirror the reference: PrefixSumKernel.ts:33-35,
README.md:97)."""
import ctypes

import pytest

from radix_sort_amd import _lib
from radix_sort_amd import RadixSortError, RadixSortKernel, PrefixSumKernel


def test_library_exports_every_header_symbol():
    L = _lib.load()
    names = _lib.header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib._SIGS, f"{n} declared in rsort.h but not bound in _lib.py"


def test_version_and_status_strings():
    L = _lib.load()
    assert L.rs_version() == (0 << 16) | 6
    assert L.rs_status_string(_lib.RS_ERR_NOT_POW2).decode().startswith("workgroup")
    assert "device-side failure" in L.rs_status_string(_lib.RS_ERR_DEVICE).decode()


def _create(**kw):
    d = dict(device=0, count=1000, bit_count=32, workgroup_x=16, workgroup_y=16, flags=0,
             radix_bits=0, usage=0)
    d.update(kw)
    desc = _lib.PlanDesc(**d)
    p = ctypes.c_void_p()
    st = _lib.load().rs_plan_create(ctypes.byref(desc), ctypes.byref(p))
    return st, p


@pytest.mark.parametrize("wx,wy", [(3, 16), (16, 12), (64, 32)])
def test_plan_rejects_bad_workgroup(wx, wy):
    st, p = _create(workgroup_x=wx, workgroup_y=wy)
    assert st == _lib.RS_ERR_NOT_POW2 and not p.value
    assert "power of two" in _lib.load().rs_last_error().decode()


@pytest.mark.parametrize("bits", [2, 6, 30, 36])
def test_plan_rejects_bad_bit_count(bits):
    st, _ = _create(bit_count=bits)
    assert st == _lib.RS_ERR_BIT_COUNT


def test_plan_rejects_bad_radix_bits_and_flags():
    assert _create(radix_bits=3)[0] == _lib.RS_ERR_INVALID_ARG
    assert _create(usage=2)[0] == _lib.RS_ERR_INVALID_ARG
    assert "usage" in _lib.load().rs_last_error().decode()
    assert _create(flags=0x100)[0] == _lib.RS_ERR_INVALID_ARG
    assert _create(count=1 << 33)[0] == _lib.RS_ERR_INVALID_ARG


def test_scan_plan_rejects_bad_workgroup():
    p = ctypes.c_void_p()
    st = _lib.load().rs_scan_plan_create(0, 10, 12, 1, 0, ctypes.byref(p))
    assert st == _lib.RS_ERR_NOT_POW2


def test_null_arguments():
    L = _lib.load()
    assert L.rs_plan_create(None, None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_plan_sort(None, None, None, None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_plan_check(None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_scan_plan_run_indirect(None, None, None, 0, None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_scan_plan_dispatch_chain(None, None, 0) == 0
    assert L.rs_plan_last_path(None, None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_plan_last_split(None, None) == _lib.RS_ERR_INVALID_ARG
    assert L.rs_plan_set_debug(None, None) == _lib.RS_ERR_INVALID_ARG
    L.rs_plan_destroy(None)  # no-op


def test_debug_struct_and_kernel_kinds_match_the_header():
    """The Python mirrors of rs_plan_debug (every field, the split switch last) and of the kernel
    kinds (RS_KERNEL_PRESORTED = 7, RS_KERNEL_KINDS = 8) agree with include/rsort.h."""
    import os
    import re
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "rsort.h")).read()
    body = hdr[hdr.index("typedef struct rs_plan_debug"):hdr.index("} rs_plan_debug;")]
    fields = re.findall(r"int32_t\s+(\w+);", body)
    assert [f for f, _ in _lib.PlanDebug._fields_] == fields
    assert fields[-1] == "high_half"
    assert re.search(r"RS_KERNEL_SPLIT = 6", hdr) and re.search(r"RS_KERNEL_PRESORTED = 7", hdr)
    assert re.search(r"RS_KERNEL_KINDS = 8", hdr)
    assert _lib.RS_KERNEL_KINDS == 8 and _lib.KERNEL_NAMES[_lib.RS_KERNEL_SPLIT] == "split"
    assert _lib.KERNEL_NAMES[_lib.RS_KERNEL_PRESORTED] == "presorted"
    assert re.search(r"RS_PATH_PRESORTED = 5", hdr) and _lib.PATH_NAMES[5] == "presorted"


def test_python_facade_validates_both_spellings():
    # raw pointers + count: validation fails before any HIP call
    with pytest.raises(RadixSortError, match="power of two"):
        RadixSortKernel(keys=0x1000, count=10, workgroup_size={"x": 3, "y": 5})
    with pytest.raises(RadixSortError, match="power of two"):
        RadixSortKernel(data={"keys": 0x1000}, count=10, workgroupSize={"x": 6, "y": 1})
    with pytest.raises(RadixSortError, match="bit_count"):
        RadixSortKernel(keys=0x1000, count=10, bit_count=10)
    with pytest.raises(RadixSortError, match="bit_count"):
        RadixSortKernel(data={"keys": 0x1000}, count=10, bitCount=7)
    with pytest.raises(RadixSortError, match="count is required"):
        RadixSortKernel(keys=0x1000)
    with pytest.raises(RadixSortError, match="power of two"):
        PrefixSumKernel(data=0x1000, count=10, workgroupSize={"x": 3, "y": 3})


def test_interleaved_flag_is_known_and_next_bit_is_not():
    # RS_FLAG_INTERLEAVED (0x10) passes option validation; 0x20 is rejected before any device work
    assert _lib.RS_FLAG_INTERLEAVED == 0x10
    assert _create(flags=0x20)[0] == _lib.RS_ERR_INVALID_ARG
