"""Prometheus text exposition of a Serve's metrics, plus a dependency-free
asyncio HTTP endpoint (GET /metrics, GET /healthz).

    server = await start_metrics_server(serve, port=9400)
    ...
    server.close(); await server.wait_closed()

Exposes the orchestrator counters (tasks, latency quantiles, queue, agents),
the engine (steps, tokens, KV blocks, prefix-cache hits, TTFT/TPOT quantiles,
HBM) and, when attached, FaultTolerance health counts.
"""
from __future__ import annotations

import asyncio
import re
from typing import Any, Dict, List, Optional, Tuple

_PREFIX = "pilottai"


def _name(*parts: str) -> str:
    return "_".join([_PREFIX] + [re.sub(r"[^a-zA-Z0-9_]", "_", p) for p in parts if p])


def _flatten(d: Dict[str, Any], prefix: Tuple[str, ...] = ()) -> List[Tuple[str, float]]:
    out = []
    for k, v in d.items():
        if isinstance(v, bool):
            out.append((_name(*prefix, k), float(v)))
        elif isinstance(v, (int, float)):
            out.append((_name(*prefix, k), float(v)))
        elif isinstance(v, dict):
            out.extend(_flatten(v, prefix + (k,)))
    return out


def metrics_text(serve, fault_tolerance=None) -> str:
    m = serve.get_metrics()
    lines = []
    name = m.get("name", "serve")
    eng = m.pop("engine", None)
    for key, val in _flatten(m):
        lines.append(f'{key}{{serve="{name}"}} {val:g}')
    if eng is not None:
        src = None
        llm = getattr(serve, "_manager_llm", None)
        e = getattr(llm, "engine", None)
        if e is not None and hasattr(e, "latency_summary"):
            src = e.latency_summary(max(0, len(e.timings) - 10000))
        for key, val in _flatten(eng, ("engine",)):
            lines.append(f'{key}{{serve="{name}"}} {val:g}')
        for key, val in (src or {}).items():
            if isinstance(val, (int, float)):
                lines.append(f'{_name("engine", key)}{{serve="{name}"}} {val:g}')
    if fault_tolerance is not None:
        h = fault_tolerance.get_health_metrics()
        for st, n in h.get("status", {}).items():
            lines.append(f'{_name("agents_health")}{{serve="{name}",status="{st}"}} {n}')
        lines.append(f'{_name("ft_replacements")}{{serve="{name}"}} {h.get("replacements", 0)}')
        lines.append(f'{_name("ft_recoveries")}{{serve="{name}"}} {h.get("recoveries", 0)}')
    return "\n".join(lines) + "\n"


async def start_metrics_server(serve, host: str = "127.0.0.1", port: int = 9400,
                               fault_tolerance=None) -> asyncio.base_events.Server:
    async def handle(reader: asyncio.StreamReader, writer: asyncio.StreamWriter):
        try:
            req = await asyncio.wait_for(reader.readline(), 5.0)
            while (await reader.readline()) not in (b"\r\n", b"\n", b""):
                pass
            path = req.split()[1].decode() if len(req.split()) > 1 else "/"
            if path.startswith("/metrics"):
                body, ctype, code = metrics_text(serve, fault_tolerance), "text/plain; version=0.0.4", "200 OK"
            elif path.startswith("/healthz"):
                ok = not getattr(serve, "_shutting_down", False)
                body, ctype, code = ("ok\n" if ok else "stopping\n"), "text/plain", ("200 OK" if ok else "503 Service Unavailable")
            else:
                body, ctype, code = "not found\n", "text/plain", "404 Not Found"
            data = body.encode()
            writer.write(f"HTTP/1.1 {code}\r\nContent-Type: {ctype}\r\nContent-Length: {len(data)}\r\n"
                         f"Connection: close\r\n\r\n".encode() + data)
            await writer.drain()
        except Exception:  # noqa: BLE001 — a bad client must not disturb the orchestrator
            pass
        finally:
            writer.close()

    return await asyncio.start_server(handle, host, port)
