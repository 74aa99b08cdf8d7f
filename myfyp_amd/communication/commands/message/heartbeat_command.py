"""``beat`` (parity: ``message/heartbeat_command.py:27-52``)."""

from myfyp_amd.communication.commands.command import Command

heartbeater_cmd_name = "beat"


class HeartbeatCommand(Command):
    """Refresh (or add, as non-direct) the sender in the neighbour table."""

    def __init__(self, heartbeat) -> None:
        self._heartbeat = heartbeat

    @staticmethod
    def get_name() -> str:
        return heartbeater_cmd_name

    def execute(self, source: str, round: int, *args, **kwargs) -> None:
        if not args:
            raise ValueError("Heartbeat without time")
        self._heartbeat.beat(source, time=float(args[0]))
