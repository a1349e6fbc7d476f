"""Read a par file with the reference's get_model and print its as_parfile(include_info=False)
(container only; tests/test_parfile.py feeds it pint_amd's own output: a par file pint_amd
writes must read back into the same reference model).  Usage: run_ref.sh check_parfile.py PAR"""
import sys

from pint.models import get_model

print(get_model(sys.argv[1]).as_parfile(include_info=False), end="")
