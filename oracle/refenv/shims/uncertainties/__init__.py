"""Minimal stand-in for uncertainties (absent here). Test infrastructure only."""


class _UFloat(float):
    def __new__(cls, v, s=0.0):
        o = float.__new__(cls, v)
        o.nominal_value = float(v)
        o.std_dev = float(s)
        o.n = o.nominal_value
        o.s = o.std_dev
        return o


def ufloat(v, s=0.0, *a, **k):
    return _UFloat(v, s)


class umath:  # noqa: N801
    pass
