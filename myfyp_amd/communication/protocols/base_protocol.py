"""Shared protocol machinery: neighbours + client + server dispatch + gossiper + heartbeater.

The reference duplicates this wiring in ``grpc/grpc_communication_protocol.py:49-263`` and
``memory/memory_communication_protocol.py:52-268``; here both transports subclass one base and only
provide a ``Neighbors`` / ``Client`` pair and a ``start_transport``/``stop_transport`` hook.

Server-side dispatch (parity: ``grpc_server.py:161-217``, ``memory_server.py:146-204``):
dedupe by hash → relay if ``ttl > 0`` (ttl-1, direct neighbours minus the source) → execute.
"""

from __future__ import annotations

import functools
import threading
from typing import Any, Callable, Dict, List, Optional, Union

from myfyp_amd.communication.commands.command import Command
from myfyp_amd.communication.commands.message.heartbeat_command import HeartbeatCommand, heartbeater_cmd_name
from myfyp_amd.communication.protocols.client import Client
from myfyp_amd.communication.protocols.communication_protocol import CommunicationProtocol
from myfyp_amd.communication.protocols.exceptions import ProtocolNotStartedError
from myfyp_amd.communication.protocols.gossiper import Gossiper
from myfyp_amd.communication.protocols.heartbeater import Heartbeater
from myfyp_amd.communication.protocols.neighbors import Neighbors
from myfyp_amd.management.logger import logger
from myfyp_amd.settings import Settings


def running(func: Callable) -> Callable:
    """Raise ``ProtocolNotStartedError`` unless the protocol is started (parity: ``@running``)."""

    @functools.wraps(func)
    def wrapper(self, *args, **kwargs):
        if not self._started:
            raise ProtocolNotStartedError("The protocol has not been started.")
        return func(self, *args, **kwargs)

    return wrapper


class BaseCommunicationProtocol(CommunicationProtocol):
    """Transport-independent part of a protocol."""

    def __init__(self, addr: str, commands: Optional[List[Command]] = None) -> None:
        self.addr = self.parse_address(addr)
        self._neighbors = self.build_neighbors(self.addr)
        self._client = self.build_client(self.addr, self._neighbors)
        self._gossiper = Gossiper(self.addr, self._client)
        self._heartbeater = Heartbeater(self.addr, self._neighbors, self._client)
        self._commands: Dict[str, Command] = {}
        self._started = False
        self._terminated = threading.Event()
        self.add_command(HeartbeatCommand(self._heartbeater))
        if commands:
            self.add_command(commands)

    # ------------------------------------------------------------------ transport hooks
    def parse_address(self, addr: str) -> str:
        return addr

    def build_neighbors(self, addr: str) -> Neighbors:
        raise NotImplementedError

    def build_client(self, addr: str, neighbors: Neighbors) -> Client:
        raise NotImplementedError

    def start_transport(self) -> None:
        raise NotImplementedError

    def stop_transport(self) -> None:
        raise NotImplementedError

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self.start_transport()
        self._started = True
        self._terminated.clear()
        self._heartbeater.start()
        self._gossiper.start()

    @running
    def stop(self) -> None:
        self._heartbeater.stop()
        self._gossiper.stop()
        self._neighbors.clear_neighbors()
        self.stop_transport()
        self._started = False
        self._terminated.set()

    def is_running(self) -> bool:
        return self._started

    def add_command(self, cmds: Union[Command, List[Command]]) -> None:
        for c in cmds if isinstance(cmds, list) else [cmds]:
            self._commands[c.get_name()] = c

    # ------------------------------------------------------------------ server-side dispatch
    def handle_message(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        """Process an incoming control message. Returns ``{}`` or ``{"error": ...}``."""
        if not self._gossiper.check_and_set_processed(msg["hash"]):
            return {}
        cmd = msg["cmd"]
        if cmd != heartbeater_cmd_name or not Settings.EXCLUDE_BEAT_LOGS:
            logger.debug(self.addr, f"📫 {cmd.upper()} received from {msg['source']} (ttl={msg['ttl']})")
        if msg["ttl"] > 0:
            relay = dict(msg, ttl=msg["ttl"] - 1)
            self._gossiper.add_message(relay, [n for n in self._neighbors.get_all(only_direct=True) if n != msg["source"]])
        handler = self._commands.get(cmd)
        if handler is None:
            logger.error(self.addr, f"Unknown command: {cmd} from {msg['source']}")
            return {"error": f"Unknown command: {cmd}"}
        try:
            handler.execute(msg["source"], msg["round"], *msg["args"])
        except Exception as e:
            text = f"Error while processing command: {cmd} {msg['args']}: {e}"
            logger.error(self.addr, text)
            return {"error": text}
        return {}

    def handle_weights(self, msg: Dict[str, Any]) -> Dict[str, Any]:
        """Process an incoming weights message (never relayed)."""
        handler = self._commands.get(msg["cmd"])
        if handler is None:
            return {"error": f"Unknown command: {msg['cmd']}"}
        try:
            handler.execute(msg["source"], msg["round"], weights=msg["weights"], contributors=msg["contributors"], num_samples=msg["weight"])
        except Exception as e:
            text = f"Error while processing model: {msg['cmd']}: {e}"
            logger.error(self.addr, text)
            return {"error": text}
        return {}

    def handshake(self, addr: str) -> bool:
        """A peer connected to us: add it as a direct neighbour (no handshake back)."""
        return self._neighbors.add(addr, non_direct=False, handshake_msg=False)

    def remote_disconnect(self, addr: str) -> None:
        self._neighbors.remove(addr, disconnect_msg=False)

    # ------------------------------------------------------------------ client API
    def build_msg(self, cmd: str, args: Optional[List[str]] = None, round: Optional[int] = None) -> Any:
        return self._client.build_message(cmd, args, round)

    def build_weights(self, cmd: str, round: int, serialized_model: Any, contributors: Optional[List[str]] = None, weight: int = 1) -> Any:
        return self._client.build_weights(cmd, round, serialized_model, contributors, weight)

    @running
    def send(self, nei: str, msg: Any, raise_error: bool = False, remove_on_error: bool = True, create_connection: bool = False) -> None:
        self._client.send(nei, msg, create_connection=create_connection, raise_error=raise_error, remove_on_error=remove_on_error)

    @running
    def broadcast(self, msg: Any, node_list: Optional[List[str]] = None) -> None:
        self._client.broadcast(msg, node_list)

    @running
    def connect(self, addr: str, non_direct: bool = False) -> bool:
        return self._neighbors.add(self.parse_address(addr), non_direct=non_direct)

    @running
    def disconnect(self, nei: str, disconnect_msg: bool = True) -> None:
        self._neighbors.remove(nei, disconnect_msg=disconnect_msg)

    def get_neighbors(self, only_direct: bool = False) -> Dict[str, Any]:
        return self._neighbors.get_all(only_direct)

    def get_address(self) -> str:
        return self.addr

    def wait_for_termination(self) -> None:
        self._terminated.wait()

    @running
    def gossip_weights(
        self,
        early_stopping_fn: Callable[[], bool],
        get_candidates_fn: Callable[[], List[str]],
        status_fn: Callable[[], Any],
        model_fn: Callable[[str], Any],
        period: Optional[float] = None,
        create_connection: bool = False,
        wait_fn: Optional[Callable[[float], None]] = None,
    ) -> None:
        if period is None:
            period = Settings.GOSSIP_MODELS_PERIOD
        self._gossiper.gossip_weights(early_stopping_fn, get_candidates_fn, status_fn, model_fn, period, create_connection, wait_fn)
