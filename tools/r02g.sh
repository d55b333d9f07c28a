#!/bin/bash
S=tools/gpu_step.sh
$S 900 r02g_pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread; [ $? = 99 ] && exit 1
$S 300 r02g_smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"; [ $? = 99 ] && exit 1
