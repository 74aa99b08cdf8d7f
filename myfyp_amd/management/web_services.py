"""REST client for the optional P2PFL web dashboard (parity: ``p2pfl/management/p2pfl_web_services.py:58-270``).

Endpoints and headers mirror the reference (``x-api-key``). Every call is best-effort: a dashboard
outage never stops learning.
"""

from __future__ import annotations

import datetime
from typing import Any, Dict, Optional


class P2pflWebServicesError(Exception):
    """Raised on non-2xx responses."""

    def __init__(self, code: int, message: str) -> None:
        super().__init__(f"{code}: {message}")
        self.code = code
        self.message = message


class P2pflWebServices:
    """Thin wrapper over ``requests`` for the dashboard API."""

    def __init__(self, url: str, key: str, timeout: float = 5.0) -> None:
        self.url = url.rstrip("/")
        self.key = key
        self.timeout = timeout
        self.node_id: Dict[str, Any] = {}

    def _headers(self) -> Dict[str, str]:
        return {"Content-Type": "application/json", "x-api-key": self.key}

    def _post(self, path: str, payload: Dict[str, Any]) -> Optional[Dict[str, Any]]:
        import requests

        resp = requests.post(f"{self.url}{path}", json=payload, headers=self._headers(), timeout=self.timeout)
        if resp.status_code >= 300:
            raise P2pflWebServicesError(resp.status_code, resp.text)
        try:
            return resp.json()
        except ValueError:
            return None

    def register_node(self, node: str, is_simulated: bool) -> None:
        out = self._post("/node", {"address": node, "is_simulated": is_simulated, "creation_date": str(datetime.datetime.now())})
        if out is not None and "node_id" in out:
            self.node_id[node] = out["node_id"]

    def unregister_node(self, node: str) -> None:
        self._post("/node/unregister", {"node_id": self.node_id.get(node, node)})

    def send_log(self, time: datetime.datetime, node: str, level: int, message: str) -> None:
        self._post("/node-log", {"time": str(time), "node_id": self.node_id.get(node, node), "level": level, "message": message})

    def send_local_metric(self, exp: str, round: int, metric: str, node: str, value: float, step: int) -> None:
        self._post(
            "/node-metric/local",
            {"exp": exp, "round": round, "metric": metric, "node_id": self.node_id.get(node, node), "value": value, "step": step},
        )

    def send_global_metric(self, exp: str, round: int, metric: str, node: str, value: float) -> None:
        self._post(
            "/node-metric/global",
            {"exp": exp, "round": round, "metric": metric, "node_id": self.node_id.get(node, node), "value": value},
        )

    def send_system_metric(self, node: str, metric: str, value: float, time: datetime.datetime) -> None:
        self._post("/node-metric/system", {"time": str(time), "metric": metric, "node_id": self.node_id.get(node, node), "value": value})

    def get_pending_actions(self) -> Any:
        raise NotImplementedError("Remote actions are not supported by the dashboard API yet.")
