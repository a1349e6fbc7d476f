"""Minimal stand-in for loguru (absent in this container). Test infrastructure only."""
import logging as _logging

_std = _logging.getLogger("pint-ref")


class _Level:
    def __init__(self, name, no):
        self.name = name
        self.no = no


class _Logger:
    def trace(self, *a, **k):
        pass

    debug = info = success = log = trace

    def warning(self, msg, *a, **k):
        _std.warning(str(msg))

    def error(self, msg, *a, **k):
        _std.error(str(msg))

    critical = exception = error

    def add(self, *a, **k):
        return 0

    def remove(self, *a, **k):
        pass

    def level(self, name, no=None, **k):
        return _Level(name, no if no is not None else 20)

    def opt(self, *a, **k):
        return self

    bind = patch = opt

    def configure(self, *a, **k):
        pass

    def disable(self, *a, **k):
        pass

    def enable(self, *a, **k):
        pass


logger = _Logger()
