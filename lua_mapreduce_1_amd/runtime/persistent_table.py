"""Distributed persistent key/value singleton (reference: mapreduce/persistent_table.lua).

``persistent_table(name, cnn_string="inproc", dbname="tmp", document="singletons")``
returns an object whose attributes are JSON-checked fields stored in the
coordinator.  ``update()`` is optimistic: local changes (``dirty``) are pushed
only if nobody changed the document since it was read (timestamp
compare-and-set, the findAndModify of persistent_table.lua:41-74), otherwise
it raises; a clean ``update()`` refreshes.  ``lock()``/``unlock()`` is a
test-and-set spin lock (0.1 s), ``read_only(True)`` forbids writes,
``drop()`` resets the document.  ``str(t)`` is the JSON of the user fields.
"""
from __future__ import annotations

import json

from .. import utils
from .cnn import cnn as cnn_cls

LOCK_SLEEP = 0.1
RESERVED = {"_id", "timestamp", "set", "update", "drop", "read_only", "dirty", "locked", "__dummy__", "lock",
            "unlock"}


class persistent_table:  # noqa: N801
    def __init__(self, name: str, cnn_string=None, dbname: str = "tmp", document: str = "singletons",
                 auth_table=None):
        if not isinstance(name, str):
            raise TypeError("First argument is a string name for the table")
        o = object.__setattr__
        o(self, "_cnn", cnn_cls(cnn_string, dbname, auth_table))
        o(self, "_name", name)
        o(self, "_document", document)
        o(self, "_dbname", dbname)
        o(self, "_dirty", False)
        o(self, "_read_only", False)
        o(self, "_locked", False)
        st, f = self._req("PT_OPEN")
        self._load(f)

    def _req(self, op, *args):
        return self._cnn.connect().request(op, self._dbname, self._document, self._name, *args)

    def _load(self, f):
        object.__setattr__(self, "_content", json.loads(f[0]))
        object.__setattr__(self, "_timestamp", int(f[1]))

    # -- methods -------------------------------------------------------------
    def update(self) -> None:
        if self._dirty:
            st, f = self._req("PT_UPDATE", 1, self._timestamp, json.dumps(self._content))
            if st != 0:
                raise RuntimeError("Impossible to update, data is not consistent")
        else:
            st, f = self._req("PT_UPDATE", 0, 0, "")
        self._load(f)
        object.__setattr__(self, "_dirty", False)

    def drop(self) -> None:
        st, f = self._req("PT_DROP")
        self._load(f)
        object.__setattr__(self, "_dirty", False)

    def set(self, tbl: dict) -> None:
        if self._read_only:
            raise RuntimeError("Unable to write in a read_only persistent table")
        for k, v in tbl.items():
            utils.assert_check(v)
            if k in RESERVED:
                raise KeyError(f"{k} field is reserved")
            self._content[k] = v
        object.__setattr__(self, "_dirty", True)

    def lock(self) -> None:
        while True:
            st, f = self._req("PT_LOCK")
            if int(f[0]) == 0:
                break
            utils.sleep(LOCK_SLEEP)
        object.__setattr__(self, "_locked", True)

    def unlock(self) -> None:
        self._req("PT_UNLOCK")
        object.__setattr__(self, "_locked", False)

    def read_only(self, v: bool) -> None:
        object.__setattr__(self, "_read_only", bool(v))

    def dirty(self) -> bool:
        return self._dirty

    # -- field access ----------------------------------------------------------
    def __getattr__(self, key):
        if key.startswith("_"):
            raise AttributeError(key)
        return self._content.get(key)

    def __setattr__(self, key, value):
        if value is None:
            self._content.pop(key, None)
            object.__setattr__(self, "_dirty", True)
        else:
            self.set({key: value})

    __getitem__ = __getattr__

    def __setitem__(self, key, value):
        self.__setattr__(key, value)

    def __str__(self) -> str:
        return json.dumps({k: v for k, v in self._content.items() if k not in RESERVED})

    def __del__(self):
        try:
            if self._locked:
                self.unlock()
        except Exception:  # noqa: BLE001
            pass


def utest(connection_string=None) -> None:
    conf = persistent_table("conf", connection_string)
    conf.drop()
    conf.set({"key": "test"})
    conf.update()
    conf2 = persistent_table("conf", connection_string)
    conf2.update()
    assert conf.key == conf2.key
