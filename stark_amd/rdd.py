"""Minimal local stand-in for the PySpark pieces stark touches (third-party in the
reference: stark/stark.py:1, 35, 65-66, 79-85; example/stark_ex.py:16-18).

Spark's role in the reference is plumbing: partition the rows, run one Stan job per
partition, bring the P x S results back to the driver and fold them with
``functools.reduce``.  Here partitions are shards that live on GPUs (one process per GPU,
``stark_amd.dist``), so only the data-partitioning semantics are kept:

  * ``parallelize(data, k)`` slices like Spark's ParallelCollectionRDD: partition i holds
    rows [i*n//k, (i+1)*n//k);
  * ``mapPartitions`` / ``reduce`` / ``coalesce(1)`` / ``union`` / ``collect`` / ``glom``
    follow PySpark semantics (reduce folds in partition order).

A real ``pyspark`` RDD also works with ``stark_amd.stark.Stark``: only
``getNumPartitions()`` and ``glom().collect()`` are used on it.
"""
from __future__ import annotations

import functools


class LocalRDD:
    def __init__(self, partitions):
        self._parts = [list(p) for p in partitions]

    def getNumPartitions(self) -> int:
        return len(self._parts)

    def glom(self):
        return LocalRDD([[list(p)] for p in self._parts])

    def collect(self):
        return [x for p in self._parts for x in p]

    def mapPartitions(self, f):
        return LocalRDD([list(f(iter(p))) for p in self._parts])

    def reduce(self, f):
        vals = self.collect()
        if not vals:
            raise ValueError("Can not reduce() empty RDD")
        return functools.reduce(f, vals)

    def coalesce(self, n: int, shuffle: bool = False):
        if n >= len(self._parts):
            return LocalRDD(self._parts)
        parts = []
        for i in range(n):
            lo, hi = i * len(self._parts) // n, (i + 1) * len(self._parts) // n
            parts.append([x for p in self._parts[lo:hi] for x in p])
        return LocalRDD(parts)

    def union(self, other):
        return LocalRDD(self._parts + other._parts)

    def partitions(self):
        return [list(p) for p in self._parts]


class LocalContext:
    """SparkContext stand-in: ``sc.parallelize(data, numSlices)``."""

    def __init__(self, appName: str = "stark_amd"):
        self.appName = appName

    def parallelize(self, data, numSlices: int = 2) -> LocalRDD:
        data = list(data)
        n = len(data)
        k = max(1, int(numSlices))
        return LocalRDD([data[i * n // k:(i + 1) * n // k] for i in range(k)])


def partitions_of(rdd):
    """Rows of every partition, for LocalRDD or a pyspark RDD."""
    if isinstance(rdd, LocalRDD):
        return rdd.partitions()
    return [list(p) for p in rdd.glom().collect()]
