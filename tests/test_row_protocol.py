"""CPU coverage of the north_star ROW layout at N>1: its round protocol
(owned rows, ghost rows of the senders by want lists, the pull-validity and
ring-target reductions, D_r's count / first-detector reductions), modelled in
numpy (tests/row_model.py) and run as world-size 2 and 3 torch.distributed
gloo groups on 127.0.0.1, must reproduce the full CPU oracle bit for bit on
every rank's rows, the counters and the failed / detector read-outs, in pull
and ring mode, under crash / leave / join churn. The HIP side runs the same
exchange set (tests/test_gpu_rows.py checks it against the oracle over the
in-process transport, G = 2..8)."""
import socket

import pytest
import torch.multiprocessing as mp

import row_model


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n,peer_mode,t_fail,churn", [
    (2, 40, 0, 5, 11), (3, 70, 0, 3, 12), (2, 40, 1, 5, 13), (3, 70, 1, 4, 14), (3, 33, 1, 2, 15)])
def test_row_protocol_matches_oracle(oracle_mod, world, n, peer_mode, t_fail, churn):
    cfg = dict(peer_mode=peer_mode, fanout=3, seed=0xA00 + churn, t_fail=t_fail, t_cleanup=5)
    mp.spawn(row_model.worker, args=(world, free_port(), n, 25, cfg, churn), nprocs=world, join=True)
