#!/bin/bash
# Round-2 final-build GPU session: host/GPU NUMA topology, smoke, the whole -m gpu suite, the default bench line.
# Each GPU step under its own time limit, chained with &&.
set -o pipefail
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"
O=gpurun_out/${1:-final}
mkdir -p $O
{
  echo "nodes: $(ls -d /sys/devices/system/node/node* | xargs -n1 basename | tr '\n' ' ')"
  for n in /sys/devices/system/node/node*; do echo "$(basename $n) cpus $(cat $n/cpulist) mem $(grep MemTotal $n/meminfo | awk '{print $4,$5}')"; done
  for d in /sys/class/drm/card*/device; do [ -f $d/numa_node ] && echo "$d numa_node=$(cat $d/numa_node) vendor=$(cat $d/vendor) dev=$(cat $d/device)"; done
  echo "allowed cpus: $(grep Cpus_allowed_list /proc/self/status)"
  echo "allowed mems: $(grep Mems_allowed_list /proc/self/status)"
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null; cat /sys/fs/cgroup/cpuset.mems.effective 2>/dev/null
  nproc
} > $O/topology.log 2>&1
cat $O/topology.log
timeout -k 10 300 python3 __graft_entry__.py smoke > $O/smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 600 python3 bench.py > $O/bench_n1.json 2> $O/bench_n1.err && echo BENCH_OK
rc=$?
tail -3 $O/smoke.log $O/pytest_gpu.log; cat $O/bench_n1.json; tail -5 $O/bench_n1.err
exit $rc
