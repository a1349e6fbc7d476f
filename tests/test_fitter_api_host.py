"""Host logic of the fitter reporting API (no GPU): the value(uncertainty) shorthand of
get_summary, and the labelled covariance / correlation matrices (pint_matrix.py:687-831)."""
import numpy as np
import pytest

from pint_amd.pint_matrix import CorrelationMatrix, CovarianceMatrix
from pint_amd.summary import shorthand


@pytest.mark.parametrize("v,u,want", [
    # the uncertainties package's documented shorthand ("S") outputs
    (0.2, 0.01, "0.200(10)"),
    (1234.56789, 0.1, "1234.57(10)"),
    (3.14159, 0.0047, "3.142(5)"),
    # Particle Data Group rounding of the uncertainty: 100-354 two digits, 355-949 one,
    # 950-999 up to two digits of the next decade
    (1.0, 0.0354, "1.000(35)"),
    (1.0, 0.0355, "1.00(4)"),
    (1.0, 0.0960, "1.00(10)"),
    # a common exponent below 1e-4
    (1.23e-8, 4.2e-10, "1.23(4)×10⁻⁸"),
    # longdouble values keep their digits
    (np.longdouble("218.811843850012345"), 1.3e-11, "218.811843850012(13)"),
])
def test_shorthand(v, u, want):
    assert shorthand(v, u) == want


def test_shorthand_no_uncertainty():
    assert shorthand(1.5, 0.0) == "1.5"
    assert shorthand(1.5, None) == "1.5"


def test_matrices():
    rng = np.random.default_rng(3)
    a = rng.normal(size=(4, 4))
    cov = a @ a.T
    names = ["Offset", "F0", "RAJ", "DECJ"]
    c = CovarianceMatrix(cov, names)
    corr = c.to_correlation_matrix()
    assert isinstance(corr, CorrelationMatrix)
    e = np.sqrt(np.diag(cov))
    assert np.allclose(corr.matrix, cov / np.outer(e, e))
    sub = c.get_label_matrix(["RAJ", "F0"])
    assert np.array_equal(sub.matrix, cov[np.ix_([2, 1], [2, 1])])
    txt = corr.prettyprint(usecolor=False)
    lines = txt.splitlines()
    assert lines[1] == "Parameter correlation matrix:"
    assert "Offset" not in txt                       # offset=False drops the phase column
    assert "Offset" in corr.prettyprint(offset=True, usecolor=False)
    first = corr.prettyprint(coordinatefirst=True, usecolor=False).splitlines()[2].split()
    assert first == ["RAJ", "DECJ", "F0"]
    # the reference's label dicts are accepted too
    lab = {n: (i, i + 1, "") for i, n in enumerate(names)}
    assert CovarianceMatrix(cov, [lab, lab]).labels == names
    with pytest.raises(ValueError):
        CovarianceMatrix(np.zeros((2, 3)), ["a", "b"])
