"""Rendezvous for the multi-process CPU tests without a port race: the test process hosts a
listening TCPStore on an ephemeral port for the whole test, and every rank joins it as a
client. (Binding port 0, closing the socket and handing the number to the ranks lets
another process take the port first: DESIGN.md §7.)"""
import datetime

import torch.distributed as dist

_TIMEOUT = datetime.timedelta(seconds=240)


def parent_store() -> dist.TCPStore:
    """The server side; keep the returned object alive until the ranks have exited."""
    return dist.TCPStore("127.0.0.1", 0, None, True, timeout=_TIMEOUT, wait_for_workers=False)


def join(rank: int, world: int, port: int, backend: str = "gloo") -> None:
    """A rank's init_process_group through the parent's store."""
    store = dist.TCPStore("127.0.0.1", port, None, False, timeout=_TIMEOUT)
    dist.init_process_group(backend, store=store, rank=rank, world_size=world)
