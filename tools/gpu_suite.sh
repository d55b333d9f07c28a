#!/bin/bash
# Full GPU parity suite + smoke (the driver's round-end checks), logs under
# gpurun_out/<tag>_*.  usage: tools/gpu_suite.sh TAG
tag=${1:?tag}
S=tools/gpu_step.sh
$S 900 ${tag}_pytest.log python -u -m pytest tests -m gpu -q --tb=line --timeout 300 --timeout-method thread; [ $? = 99 ] && exit 1
$S 300 ${tag}_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"; [ $? = 99 ] && exit 1
exit 0
