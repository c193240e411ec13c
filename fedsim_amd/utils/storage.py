"""Key -> object store with read/write-protection warnings.

Same contract as the reference's ``Storage`` (fedsim/utils/storage.py:7-130):
``read`` of a missing key returns None; protected entries only print warnings.
The server epilogue reads ``cloud_params``, ``optimizer``, ``lr_scheduler``,
``avg_params`` and ``beta`` from it (fedavg.py:196-198, adabest.py:174-182).
"""
from __future__ import annotations


class Storage(object):
    def __init__(self) -> None:
        self._storage = dict()

    def write(self, key, obj, read_protected=False, write_protected=False, silent=False):
        prev = self._storage.get(key)
        if prev is not None and prev[2] and not silent:
            print(f"Warning: write protected entry {key} is over-written")
        self._storage[key] = (obj, read_protected, write_protected)

    def read(self, key, silent=False):
        entry = self._storage.get(key)
        if entry is None:
            return None
        obj, read_p, _ = entry
        if read_p and not silent:
            print(f"Warning: read access to read-protected entry {key}")
        return obj

    def get_all_keys(self):
        return self._storage.keys()

    def get_keys(self):
        return [k for k, (_, r_p, _) in self._storage.items() if not r_p]

    def change_protection(self, key, read_protected=False, write_protected=False, silent=False):
        if key not in self._storage:
            raise Exception(f"key {key} not in storage.")
        obj, r_p, w_p = self._storage[key]
        if not silent and r_p and not read_protected:
            print(f"read protection removed from storage entry {key}.")
        if not silent and w_p and not write_protected:
            print(f"write protection removed from storage entry {key}.")
        self._storage[key] = (obj, read_protected, write_protected)

    def get_protection_status(self, key):
        if key not in self._storage:
            raise Exception(f"key {key} not in storage.")
        _, r_p, w_p = self._storage[key]
        return r_p, w_p

    def remove(self, key, silent=False):
        if key not in self._storage:
            raise Exception(f"key {key} not in storage.")
        if not silent and self._storage[key][2]:
            print(f"write protected entry {key} is removed from the storage.")
        del self._storage[key]
