"""Stand-in for numdifftools: every entry point raises. Test infrastructure only."""


class _Missing:
    def __init__(self, *a, **k):
        raise NotImplementedError("numdifftools is not available in this container")


Hessian = Derivative = Gradient = Jacobian = MaxStepGenerator = _Missing
