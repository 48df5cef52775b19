"""TEST INFRASTRUCTURE: an oracle-backed stand-in for one band handle, with
the OccupancyMapper methods the sharded layer (dm/sharded.py) calls, so the
multi-rank merge logic can be tested with gloo on CPU."""
import numpy as np

import oracle
from dm.grid import Frontiers


class OracleBand:
    def __init__(self, params):
        self.om = oracle.OracleMap(params)
        self.halo = (None, None)
        self._edges = None

    def integrate(self, poses, ranges, amin, inc):
        return self.om.integrate(poses, ranges, amin, inc)

    def edge_rows(self):
        return self.om.state[0].copy(), self.om.state[-1].copy()

    def set_halo(self, before=None, after=None):
        self.halo = (before, after)

    def frontiers(self, want_mask=False, want_labels=False):
        mask, labels, clusters = self.om.frontiers(*self.halo)
        self._edges = (labels[0].copy(), labels[-1].copy())
        return Frontiers(clusters=clusters, mask=mask if want_mask else None,
                         labels=labels if want_labels else None)

    def edge_labels(self):
        return self._edges

    def close(self):
        pass
