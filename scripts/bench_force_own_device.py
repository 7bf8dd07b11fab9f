#!/usr/bin/env python
"""bench.py with the fit's side-stream fetch overlap forced on (models/gbdt.py _own_device -> True) even
when ranks share the GPU: a rehearsal, on the one-GPU pool, of the data-parallel path an 8-GPU node takes
(two grow calls, the first part's trees fetched on a side stream while the last 32 grow). Diagnosis only."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cobalt_smart_lender_ai_amd.models.gbdt as gbdt  # noqa: E402

gbdt._own_device = lambda world: True
sys.argv[0] = "bench.py"
runpy.run_path("bench.py", run_name="__main__")
