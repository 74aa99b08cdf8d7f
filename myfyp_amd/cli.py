"""Command-line interface (parity: ``p2pfl/cli.py:65-238``).

    python -m myfyp_amd experiment list
    python -m myfyp_amd experiment run mnist --nodes 4 --rounds 3 --protocol memory
    python -m myfyp_amd experiment help mnist
    python -m myfyp_amd run myfyp_amd/examples/configs/mnist_fedavg_memory.yaml
    python -m myfyp_amd launch --address 127.0.0.1:6666        # one gRPC node, Ctrl-C to stop
    python -m myfyp_amd login / remote                           # not implemented (as in the reference)

Examples are the ``*.py`` files of :mod:`myfyp_amd.examples`; ``run`` streams the child process'
output and propagates its exit code (the reference swallows failures, ``cli.py:214-217``).
"""

from __future__ import annotations

import os
import subprocess
import sys
import time
from typing import Dict, List, Optional

import typer
from rich.console import Console
from rich.panel import Panel
from rich.table import Table

console = Console()
app = typer.Typer(help="myfyp_amd | decentralized federated learning on MI355X", no_args_is_help=True, add_completion=False)
exp_app = typer.Typer(help="Run bundled example experiments.", no_args_is_help=True)
app.add_typer(exp_app, name="experiment")

EXAMPLES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "examples")


def _read_docstring(path: str) -> str:
    with open(path) as f:
        parts = f.read().split('"""')
    return parts[1].strip() if len(parts) > 1 else ""


def available_examples() -> Dict[str, str]:
    files = sorted(f[:-3] for f in os.listdir(EXAMPLES_DIR) if f.endswith(".py") and not f.startswith("__"))
    return {f: _read_docstring(os.path.join(EXAMPLES_DIR, f + ".py")) for f in files}


def _check(example: str) -> str:
    if example not in available_examples():
        console.print(Panel(f"Example [bold yellow]{example}[/] not found. Use [bold green]experiment list[/].", title="[red]Example Not Found"))
        raise typer.Exit(code=1)
    return os.path.join(EXAMPLES_DIR, example + ".py")


@app.command()
def login(token: str = typer.Option("", help="API token")) -> None:
    """Authenticate with a remote platform (not implemented, as in the reference)."""
    console.print("[yellow]Not implemented yet.[/]")


@app.command()
def remote() -> None:
    """Interact with a remote node (not implemented, as in the reference)."""
    console.print("[yellow]Not implemented yet.[/]")


@app.command()
def launch(
    address: str = typer.Option("127.0.0.1:6666", help="listen address (host:port or unix:///path)"),
    connect: List[str] = typer.Option([], help="peer address to connect to (repeatable)"),
    rounds: int = typer.Option(0, help="start learning with this many rounds (0 = just serve)"),
    epochs: int = typer.Option(1),
    duration: float = typer.Option(0.0, help="stop after this many seconds (0 = until Ctrl-C)"),
) -> None:
    """Launch one gRPC node with the MNIST MLP on a synthetic partition (the reference's stub)."""
    from myfyp_amd.communication.protocols.grpc.grpc_communication_protocol import GrpcCommunicationProtocol
    from myfyp_amd.learning.dataset.synthetic import synthetic_mnist
    from myfyp_amd.learning.frameworks.torch import TorchModel
    from myfyp_amd.models import MLP
    from myfyp_amd.node import Node

    node = Node(TorchModel(MLP()), synthetic_mnist(6000, 1000), address=address, protocol=GrpcCommunicationProtocol)
    node.start()
    console.print(f"node listening at [bold]{node.addr}[/]")
    try:
        for peer in connect:
            node.connect(peer)
        if rounds > 0:
            time.sleep(1.0)
            node.set_start_learning(rounds=rounds, epochs=epochs)
        t0 = time.time()
        while duration <= 0 or time.time() - t0 < duration:
            time.sleep(0.2)
            if rounds > 0 and node.learning_workflow.finished and node.state.round is None:
                break
    except KeyboardInterrupt:
        pass
    finally:
        node.stop()


@app.command("run")
def run_config(config: str = typer.Argument(..., help="YAML experiment file")) -> None:
    """Run a YAML-described experiment (see myfyp_amd/examples/configs). Under ``torchrun`` each
    rank hosts its share of the peers (collective protocol) and rank 0 prints the merged results."""
    from myfyp_amd.runner import run_experiment

    if not os.path.exists(config):
        console.print(f"[red]No such file: {config}")
        raise typer.Exit(code=1)
    res = run_experiment(config)
    if res.get("world", 1) > 1:
        from myfyp_amd.parallel.federation import Federation

        Federation.get().shutdown()


@exp_app.command("list")
def list_examples() -> None:
    """List available examples."""
    table = Table(title="Available Examples", show_lines=True, expand=True, header_style="bold magenta")
    table.add_column("Name", style="green", width=14)
    table.add_column("Description")
    for name, desc in available_examples().items():
        table.add_row(name, desc)
    console.print(table)


@exp_app.command("run", context_settings={"allow_extra_args": True, "ignore_unknown_options": True})
def run_example(ctx: typer.Context, example: str) -> None:
    """Run an example; extra arguments are passed through."""
    path = _check(example)
    console.print(f"[bold yellow]Running example {example}...[/]\n")
    proc = subprocess.Popen([sys.executable, path] + list(ctx.args), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, bufsize=1, text=True)
    assert proc.stdout is not None
    for line in proc.stdout:
        print(line, end="")
    rc = proc.wait()
    if rc != 0:
        console.print(f"\n[bold red]Error running {example} (exit {rc})[/]")
        raise typer.Exit(code=rc)
    console.print(f"\n[bold green]Example {example} completed![/]")


@exp_app.command("help")
def help_example(example: str) -> None:
    """Show the --help of an example."""
    path = _check(example)
    res = subprocess.run([sys.executable, path, "--help"], capture_output=True, text=True)
    if res.returncode != 0:
        console.print(f"[red]Error running {example} --help[/]\n{res.stderr}")
        raise typer.Exit(code=1)
    console.print(Panel(res.stdout, title=f"[bold green]{example} Help"))


def main(argv: Optional[List[str]] = None) -> None:
    app(args=argv)


if __name__ == "__main__":
    main()
