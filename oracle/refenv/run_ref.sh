#!/bin/bash
# Run a script against the read-only reference (container only; test-infrastructure).
HERE="$(cd "$(dirname "$0")" && pwd)"
exec env -i PATH=/opt/conda/bin:/usr/bin:/bin HOME="$HERE/home" \
  PYTHONPATH="$HERE/shims:/root/reference/src" PYTHONDONTWRITEBYTECODE=1 PYTHONHASHSEED="${PYTHONHASHSEED:-random}" \
  /opt/conda/bin/python3.9 -W ignore "$@"
