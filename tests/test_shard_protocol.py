"""CPU coverage of the multi-GPU path (N>1): the column-sharded round
protocol of the HIP engine, modelled in numpy (tests/shard_model.py) and run
as world-size 2 and 3 torch.distributed gloo groups on 127.0.0.1, must
reproduce the full CPU oracle bit for bit on every rank's column slice, the
counters and the failed/detector read-outs, in pull and ring mode, under
crash/leave/join churn. The same exchange set runs over RCCL on the GPUs
(tests/test_gpu_sharded.py checks the HIP side against the oracle)."""
import socket

import pytest
import torch.multiprocessing as mp

import shard_model


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n,peer_mode,t_fail,churn", [
    (2, 40, 0, 5, 1), (2, 40, 1, 5, 2), (3, 70, 0, 3, 3), (3, 70, 1, 4, 4), (2, 33, 1, 2, 5)])
def test_sharded_protocol_matches_oracle(oracle_mod, world, n, peer_mode, t_fail, churn):
    cfg = dict(peer_mode=peer_mode, fanout=3, seed=0x900 + churn, t_fail=t_fail, t_cleanup=5)
    mp.spawn(shard_model.worker, args=(world, free_port(), n, 25, cfg, churn, {5, 20}), nprocs=world, join=True)
