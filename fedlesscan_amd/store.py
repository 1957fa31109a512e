"""In-memory stand-ins for the reference's MongoDB/GridFS DAOs on the hot path.

MongoDB itself is out of scope.  What the aggregation path
depends on is *which* results are selected, in *which order*, and the counts
reported afterwards; those semantics are restated here:

  ClientResultDao.save                     client_daos.py:47-90   (upsert on (session, round, client))
  ClientResultDao._retrieve_result_files   client_daos.py:125-147 (lazy iterator over the dicts)
  ClientResultDao.load_results_for_round   client_daos.py:150-162 (round_id == R)
  ClientResultDao.load_results_for_session client_daos.py:165-180 (round_id >= R - tolerance)
  delete_results_for_round / _for_session  client_daos.py:183-219
  count_results_for_round / _for_session   client_daos.py:221-235 (session count = ALL session docs)
  ParameterDao.save / load / load_latest   client_daos.py:351-437

Iteration order is insertion order; an upsert of an existing
(session, round, client) key keeps its position (Mongo natural order keeps a
replaced document's record slot).

Each stored result is what GridFS holds in the reference: the BSON bytes of
`result.dict()` (client_daos.py:73, 369), written by fedlesscan_amd.bsondoc.
Loading parses them back (client_daos.py:142, 397); results come back with the
NPZ blob as a zero-copy view into those bytes, so the ingest never copies it.
With pinned=True the documents are written into page-locked memory
(fedlesscan_amd.pinned, needs a GPU): the ingest then DMAs every layer straight
from the document to the device, with no host-side packing copy.
"""
from __future__ import annotations

import itertools
import threading
from typing import Dict, Iterator, List, Optional, Tuple

from . import bsondoc
from .common.models import ClientResult, SerializedParameters


class DocumentNotLoadedException(Exception):
    pass


class InMemoryClientResultStore:
    def __init__(self, pinned: bool = False):
        self._docs: List[dict] = []
        self._files: Dict[int, bytes] = {}  # file_id -> BSON document (the GridFS file; pinned: a memoryview)
        self.pinned = pinned
        self._ids = itertools.count(1)
        self._lock = threading.Lock()

    def save(self, session_id: str, round_id: int, client_id: str, result, overwrite: bool = True):
        # client_daos.py:55-56, 73: a ClientResult is dumped, a dict is stored as given
        doc = result.model_dump() if isinstance(result, ClientResult) else result
        if self.pinned:
            from .pinned import pinned_bytes
            data = bsondoc.encode_into(doc, pinned_bytes)
        else:
            data = bsondoc.encode(doc)
        with self._lock:
            key = (session_id, round_id, client_id)
            existing = next((d for d in self._docs
                             if (d["session_id"], d["round_id"], d["client_id"]) == key), None)
            if existing is not None and not overwrite:
                raise ValueError(f"Client result for session {session_id} and round {round_id} for client "
                                 f"{client_id} already exists. Force overwrite with overwrite=True")
            file_id = next(self._ids)
            self._files[file_id] = data
            doc = {"session_id": session_id, "round_id": round_id, "client_id": client_id, "file_id": file_id}
            if existing is not None:
                self._files.pop(existing["file_id"], None)
                existing.clear()
                existing.update(doc)
            else:
                self._docs.append(doc)

    def load(self, session_id: str, round_id: int, client_id: str) -> ClientResult:
        for d in self._docs:
            if (d["session_id"], d["round_id"], d["client_id"]) == (session_id, round_id, client_id):
                return bsondoc.client_result_from_bson(self._files[d["file_id"]])
        raise DocumentNotLoadedException(
            f"Client result for session {session_id} and round {round_id} for client {client_id} not found.")

    def _retrieve(self, dicts: List[dict], session_id: str, round_id: int) -> Iterator[ClientResult]:
        for d in dicts:
            f = self._files.get(d["file_id"])
            if f is None:
                raise DocumentNotLoadedException(
                    f"GridFS file with results in session {session_id},{round_id} and client round "
                    f"{d['round_id']} not found.")
            yield bsondoc.client_result_from_bson(f)

    def load_results_for_round(self, session_id: str, round_id: int) -> Tuple[List[dict], Iterator[ClientResult]]:
        dicts = [dict(d) for d in self._docs if d["session_id"] == session_id and d["round_id"] == round_id]
        return dicts, self._retrieve(dicts, session_id, round_id)

    def load_results_for_session(self, session_id: str, round_id: int, tolerance: int):
        dicts = [dict(d) for d in self._docs
                 if d["session_id"] == session_id and d["round_id"] >= round_id - tolerance]
        return dicts, self._retrieve(dicts, session_id, round_id)

    def delete_results_for_round(self, session_id: str, round_id: int):
        with self._lock:
            keep = []
            for d in self._docs:
                if d["session_id"] == session_id and d["round_id"] == round_id:
                    self._files.pop(d["file_id"], None)
                else:
                    keep.append(d)
            self._docs = keep

    def delete_results_for_session(self, session_id: str):
        with self._lock:
            keep = []
            for d in self._docs:
                if d["session_id"] == session_id:
                    self._files.pop(d["file_id"], None)
                else:
                    keep.append(d)
            self._docs = keep

    def count_results_for_round(self, session_id: str, round_id: int) -> int:
        return sum(1 for d in self._docs if d["session_id"] == session_id and d["round_id"] == round_id)

    def count_results_for_session(self, session_id: str) -> int:
        return sum(1 for d in self._docs if d["session_id"] == session_id)


class InMemoryParameterStore:
    """ParameterDao (client_daos.py:351-437): global model blob per (session, round)."""

    def __init__(self):
        self._params: Dict[Tuple[str, int], bytes] = {}  # (session, round) -> BSON document

    def save(self, session_id: str, round_id: int, params: SerializedParameters, overwrite: bool = True):
        key = (session_id, round_id)
        if key in self._params and not overwrite:
            raise ValueError(f"Parameters for session {session_id} and round {round_id} already exist")
        self._params[key] = bsondoc.encode(params.model_dump())

    def load(self, session_id: str, round_id: int) -> SerializedParameters:
        try:
            data = self._params[(session_id, round_id)]
        except KeyError:
            raise DocumentNotLoadedException(f"Parameters for session {session_id} round {round_id} not found")
        return bsondoc.parameters_from_bson(data)

    def load_latest(self, session_id: str) -> SerializedParameters:
        rounds = [r for (s, r) in self._params if s == session_id]
        if not rounds:
            raise DocumentNotLoadedException(f"No parameters for session {session_id}")
        return self.load(session_id, max(rounds))

    def get_latest_round(self, session_id: str) -> Optional[int]:
        rounds = [r for (s, r) in self._params if s == session_id]
        return max(rounds) if rounds else None
