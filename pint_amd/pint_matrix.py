"""Labelled parameter covariance / correlation matrices of a fit (host mirror of the
reference's ``pint_matrix.py:687-831`` CovarianceMatrix / CorrelationMatrix).

The fitters hand out the timing-parameter block (the columns of ``model.free_params`` plus
the implicit Offset, in design-matrix order).  The reference's GLSFitter matrix also carries
unlabelled rows for the noise-basis amplitudes (``fitter.py:2234-2252``); its labelled part
is this block.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np


def _colorize(text, color, attribute=None):
    """ANSI colour codes as the reference's ``plot_utils.colorize``."""
    codes = {"green": 32, "yellow": 33, "red": 31}
    pre = "\033[" + (("7;" if attribute == "reverse" else "") + str(codes[color])) + "m"
    return pre + text + "\033[0m"


class CovarianceMatrix:
    """A symmetric matrix with one label per row/column (pint_matrix.py:687)."""

    matrix_type = "covariance"

    def __init__(self, matrix, labels: Sequence):
        matrix = np.asarray(matrix)
        if matrix.ndim != 2 or matrix.shape[0] != matrix.shape[1]:
            raise ValueError("The input matrix is not symmetric.")
        if labels and isinstance(labels[0], dict):  # the reference's [{name: (i, i+1, unit)}] * 2
            d = labels[0]
            labels = [k for k, _ in sorted(d.items(), key=lambda kv: kv[1][0])]
        self.matrix = matrix
        self.labels: List[str] = list(labels)
        if len(self.labels) != matrix.shape[0]:
            raise ValueError(f"{len(self.labels)} labels for a {matrix.shape[0]}-square matrix")

    @property
    def shape(self):
        return self.matrix.shape

    def diag(self):
        return np.diag(self.matrix)

    def get_label_names(self, axis=0):
        return list(self.labels)

    def get_label_matrix(self, labels):
        """The sub-matrix of the given labels, in that order (pint_matrix.py:271)."""
        idx = [self.labels.index(l) for l in labels]
        return type(self)(self.matrix[np.ix_(idx, idx)], list(labels))

    def to_correlation_matrix(self):
        """Divide through by sqrt(diag) (pint_matrix.py:812)."""
        e = np.sqrt(self.diag())
        with np.errstate(invalid="ignore", divide="ignore"):  # a dropped (degenerate) direction: NaN, as numpy gives
            return CorrelationMatrix((self.matrix / e).T / e, self.labels)

    def _colorize_from_value(self, x, base):
        a = abs(x)
        if a < 0.5:
            return base
        if a < 0.9:
            return _colorize(base, "green")
        if a < 0.99:
            return _colorize(base, "yellow")
        if a < 0.999:
            return _colorize(base, "red")
        return _colorize(base, "red", attribute="reverse")

    def prettyprint(self, prec=3, coordinatefirst=False, offset=False, usecolor=True):
        """The labelled lower triangle as text (pint_matrix.py:723-806, same layout)."""
        fps = self.get_label_names()
        if coordinatefirst:
            coords = ["RAJ", "DECJ"] if ("RAJ" in fps and "DECJ" in fps) else (
                ["ELONG", "ELAT"] if ("ELONG" in fps and "ELAT" in fps) else [])
            if coords:
                head = ["Offset"] if "Offset" in fps else []
                fps = head + coords + [p for p in fps if p not in head + coords]
        if not offset:
            fps = [p for p in fps if p != "Offset"]
        cm = self.get_label_matrix(fps).matrix
        if self.matrix_type == "covariance":
            base = "{0: {width}.{prec}e}"
            lens = [max(len(fp) + 2, prec + 8) for fp in fps]
        else:
            base = "{0: {width}.{prec}f}"
            lens = [max(len(fp) + 2, prec + 4) for fp in fps]
        maxlen = max(lens) if lens else 0
        sout = f"\nParameter {self.matrix_type} matrix:\n"
        line = "{0:^{width}}".format("", width=maxlen)
        for fp, ln in zip(fps, lens):
            line += "{0:^{width}}".format(fp, width=ln)
        sout += line + "\n"
        for ii, fp1 in enumerate(fps):
            line = "{0:^{width}}".format(fp1, width=maxlen)
            for jj, ln in enumerate(lens[: ii + 1]):
                x = cm[ii, jj]
                text = self._colorize_from_value(x, base) if usecolor and ii != jj else base
                line += text.format(x, width=ln, prec=prec)
            sout += line + "\n"
        return sout + "\n"

    def __repr__(self):
        return self.prettyprint()


class CorrelationMatrix(CovarianceMatrix):
    """pint_matrix.py:826: the same matrix class, printed as a correlation matrix."""

    matrix_type = "correlation"
