"""A stand-in for the gossipsim package with the Engine surface bench.py
uses, for the CPU test of bench.py's argument and JSON plumbing at
--gpus > 1 (tests/test_bench_plumbing.py). It computes nothing: step()
returns fixed counters and read_timing() a fixed 1.5 ms per launch. It is
injected into sys.modules by tests/benchfake/rank.py only; the product
package never imports it."""
GH_COMM_RCCL, GH_COMM_LOCAL = 0, 1
GH_PEER_PULL, GH_PEER_RING = 0, 1
GH_DETECT_CANONICAL, GH_DETECT_QUIRK = 0, 1
GH_LAYOUT_COLUMNS, GH_LAYOUT_ROWS = 0, 1


class Config:
    def __init__(self, n, **kw):
        self.n_members = n
        self.max_files = 0
        self.__dict__.update(kw)


def default_config(n, **kw):
    return Config(n, **kw)


def comm_unique_id():
    return b"fake-comm-id"


class Engine:
    def __init__(self, cfg, rank=0, world=1, transport=None, comm_id=None):
        assert world == 1 or (comm_id == b"fake-comm-id" and transport == GH_COMM_RCCL)
        self.cfg, self.rank, self.world = cfg, rank, world
        self.n = cfg.n_members
        self.rows = cfg.shard_layout == GH_LAYOUT_ROWS
        ncs = -(-self.n // world)
        self.c0 = 0 if self.rows else rank * ncs
        self.ncol = self.n if self.rows else min(ncs, self.n - self.c0)
        self.launches = 0
        self.timing = False

    def shard_info(self):
        return self.rank, self.world, self.c0, self.ncol

    def plane_info(self):
        return 1, 1, 0

    def tier_info(self, full=False):
        return (1, 1, 0, 3) if full else (1, 1, 0)

    def init_full(self, hb0=2, ts0=0, round_=0):
        pass

    def step(self, rounds=1):
        if self.timing:
            self.launches += rounds
        return {"rounds": rounds, "detections": 0, "active_rows": self.n * rounds}

    def set_timing(self, enable=True):
        self.timing = enable

    def read_timing(self):
        return 1.5 * self.launches, self.launches

    def sync(self):
        pass

    def exchange_info(self):
        return {"ghost_rows": 22000, "bytes_out": 700 << 20, "bytes_in": 720 << 20}

    def memory_info(self):
        return {"device_bytes": 1 << 30, "wide_used": 0, "wide_cap": 1024, "frozen_rows": 0}

    def close(self):
        pass
