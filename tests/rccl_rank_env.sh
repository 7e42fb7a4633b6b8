#!/bin/bash
# Test launcher for RCCL multi-rank runs on a one-GPU box: RCCL refuses two ranks of one host on one device, so each
# rank gets its own NCCL_HOSTID (RCCL then connects the ranks over its socket transport on the loopback interface).
# Sets the environment and runs the command, before anything has touched the GPU.
export NCCL_HOSTID="msplit-test-rank${LOCAL_RANK:-${PMI_RANK:-0}}" NCCL_SOCKET_IFNAME=lo NCCL_IB_DISABLE=1
exec "$@"
