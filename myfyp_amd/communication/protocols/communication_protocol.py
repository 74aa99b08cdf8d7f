"""Transport-agnostic protocol contract (parity: ``protocols/communication_protocol.py:27-198``)."""

from abc import ABC, abstractmethod
from typing import Any, Callable, Dict, List, Optional, Union

from myfyp_amd.communication.commands.command import Command


class CommunicationProtocol(ABC):
    """What stages, commands and the Node need from a transport."""

    #: workflow implementation the node should run on top of this protocol (gossip by default)
    workflow: str = "gossip"

    @abstractmethod
    def __init__(self, addr: str = "address", commands: Optional[List[Command]] = None) -> None: ...

    @abstractmethod
    def start(self) -> None: ...

    @abstractmethod
    def stop(self) -> None: ...

    @abstractmethod
    def add_command(self, cmds: Union[Command, List[Command]]) -> None: ...

    @abstractmethod
    def build_msg(self, cmd: str, args: Optional[List[str]] = None, round: Optional[int] = None) -> Any: ...

    @abstractmethod
    def build_weights(self, cmd: str, round: int, serialized_model: bytes, contributors: Optional[List[str]] = None, weight: int = 1) -> Any: ...

    @abstractmethod
    def send(self, nei: str, msg: Any, raise_error: bool = False, remove_on_error: bool = True, create_connection: bool = False) -> None: ...

    @abstractmethod
    def broadcast(self, msg: Any, node_list: Optional[List[str]] = None) -> None: ...

    @abstractmethod
    def connect(self, addr: str, non_direct: bool = False) -> bool: ...

    @abstractmethod
    def disconnect(self, nei: str, disconnect_msg: bool = True) -> None: ...

    @abstractmethod
    def get_neighbors(self, only_direct: bool = False) -> Dict[str, Any]: ...

    @abstractmethod
    def get_address(self) -> str: ...

    @abstractmethod
    def wait_for_termination(self) -> None: ...

    @abstractmethod
    def gossip_weights(
        self,
        early_stopping_fn: Callable[[], bool],
        get_candidates_fn: Callable[[], List[str]],
        status_fn: Callable[[], Any],
        model_fn: Callable[[str], Any],
        period: Optional[float] = None,
        create_connection: bool = False,
        wait_fn: Optional[Callable[[float], None]] = None,
    ) -> None: ...
