"""Run pytest against a probe build of libsbk.so (never the product):
    SBK_PROBE_LIB=gpurun_probe_X.so python scripts/probe_pytest.py <pytest args>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import speechbrain_amd._lib as _L  # noqa: E402
_L.LIB_PATH = os.path.abspath(os.environ["SBK_PROBE_LIB"])
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[1:]))
