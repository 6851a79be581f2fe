"""Server address resolution (the reference's ``ServerConfigManager`` in
resolve_server_config.rs:30-44 was all ``todo!()``).

Resolves the three endpoints (training server, trajectory server, agent listener) from
config + constructor overrides, normalises ``*`` / ``localhost`` for bind vs connect,
and can pick free ports for tests / multi-tenant hosts.
"""
from __future__ import annotations

import socket
from dataclasses import dataclass
from typing import Dict, Optional

from ..config import ConfigLoader


@dataclass
class Endpoint:
    prefix: str
    host: str
    port: str

    def bind_address(self) -> str:
        h = "0.0.0.0" if self.host in ("*", "") else self.host
        return f"{self.prefix}{h}:{self.port}"

    def connect_address(self) -> str:
        h = "127.0.0.1" if self.host in ("*", "0.0.0.0", "", "localhost") else self.host
        return f"{self.prefix}{h}:{self.port}"

    def hostport(self) -> str:
        return f"{self.host}:{self.port}"


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


class ServerConfigManager:
    def __init__(self, config_path: Optional[str] = None, overrides: Optional[Dict[str, Dict[str, str]]] = None):
        self.cfg = ConfigLoader(None, config_path)
        self._eps = {
            "training_server": Endpoint(**self.cfg.get_train_server()),
            "trajectory_server": Endpoint(**self.cfg.get_traj_server()),
            "agent_listener": Endpoint(**self.cfg.get_agent_listener()),
        }
        for name, ov in (overrides or {}).items():
            ep = self._eps[name]
            for k, v in ov.items():
                if v is not None:
                    setattr(ep, k, str(v))

    def get(self, name: str) -> Endpoint:
        return self._eps[name]

    def assign_free_ports(self):
        for ep in self._eps.values():
            ep.port = str(free_port())
        return self

    def as_dict(self) -> Dict[str, Dict[str, str]]:
        return {k: {"prefix": e.prefix, "host": e.host, "port": e.port} for k, e in self._eps.items()}
