"""Element formats (microxscaling/mx/formats.py:12-125): enums and parameters."""
from enum import Enum, IntEnum

FP32_EXPONENT_BIAS = 127
FP32_MIN_NORMAL = 2 ** (-FP32_EXPONENT_BIAS + 1)


class RoundingMode(IntEnum):
    nearest = 0
    floor = 1
    even = 2

    @staticmethod
    def string_enums():
        return [s.name for s in RoundingMode]


class ElemFormat(Enum):
    int8 = 1
    int4 = 2
    int2 = 3
    fp8_e5m2 = 4
    fp8_e4m3 = 5
    fp6_e3m2 = 6
    fp6_e2m3 = 7
    fp4 = 8
    fp4_e2m1 = 8
    float16 = 9
    fp16 = 9
    bfloat16 = 10
    bf16 = 10

    @staticmethod
    def from_str(s):
        assert s is not None, "String elem_format == None"
        s = s.lower()
        if hasattr(ElemFormat, s):
            return getattr(ElemFormat, s)
        raise Exception("Undefined elem format", s)


def _get_min_norm(ebits):
    return 0 if ebits == 0 else 2 ** (2 - 2 ** (ebits - 1))


def _get_max_norm(ebits, mbits):
    assert ebits >= 5, "invalid for floats that don't define NaN"
    emax = 0 if ebits == 0 else 2 ** (ebits - 1) - 1
    return 2 ** emax * float(2 ** (mbits - 1) - 1) / 2 ** (mbits - 2)


# fmt -> (ebits, mbits incl. sign+implicit, emax)
_PARAMS = {
    ElemFormat.int8: (0, 8, 0), ElemFormat.int4: (0, 4, 0), ElemFormat.int2: (0, 2, 0),
    ElemFormat.fp8_e5m2: (5, 4, 15), ElemFormat.fp8_e4m3: (4, 5, 8), ElemFormat.fp6_e3m2: (3, 4, 4),
    ElemFormat.fp6_e2m3: (2, 5, 2), ElemFormat.fp4: (2, 3, 2), ElemFormat.float16: (5, 12, 15),
    ElemFormat.bfloat16: (8, 9, 127),
}


def _get_format_params(fmt):
    """(ebits, mbits, emax, max_norm, min_norm) as formats.py:61-125."""
    if isinstance(fmt, str):
        fmt = ElemFormat.from_str(fmt)
    if fmt not in _PARAMS:
        raise Exception("Unknown element format %s" % fmt)
    ebits, mbits, emax = _PARAMS[fmt]
    if fmt == ElemFormat.fp8_e4m3:
        max_norm = 2 ** emax * 1.75
    else:
        max_norm = 2 ** emax * float(2 ** (mbits - 1) - 1) / 2 ** (mbits - 2)
    return ebits, mbits, emax, max_norm, _get_min_norm(ebits)


# integer MX formats run on the device; the float element formats are outside this build's scope
INT_MBITS = {ElemFormat.int8: 8, ElemFormat.int4: 4, ElemFormat.int2: 2}
