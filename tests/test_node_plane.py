"""Node-global control plane for agent-DP (parallel/node_plane.py), multi-process on the CPU.

One process per rank (as on an 8-GPU node, minus the engines): rank 0 runs the single
manager Serve over the node-wide agent pool, the other ranks host worker agents behind
the TCP control plane. Model-free schema LLMs keep it fast; the scenarios are
parallel/node_rehearsal.py's.
"""
import pytest

from pilottai_amd.parallel.node_rehearsal import run


@pytest.mark.parametrize("world", [4, 8])
def test_skewed_submission_is_balanced_over_ranks(world):
    """Half the tasks submitted at rank 0, half at the last rank (forwarded to the manager):
    one wave of exactly one task per agent lands one task per agent, i.e. the per-rank
    counts differ by at most one; the manager's own LLM calls are spread over the ranks."""
    r = run(world, "balance", per_rank=2)
    assert r["exitcodes"] == [0] * world, r
    assert r["succeeded"] == r["submitted"] == 2 * world
    assert r["unique_completed"] == r["submitted"]
    per_rank = [r["local_executed"]] + [x["executed"] for x in r["ranks"]]
    assert len(per_rank) == world
    assert max(per_rank) - min(per_rank) <= 1, per_rank
    assert r["ranks"][-1]["forwarded_ok"] == world  # the forwarded half all came back
    # the manager's per-rank execution count (NodeManager.executions_by_rank) agrees with what
    # every rank itself executed
    assert [r["executions_by_rank"][str(k)] for k in range(world)] == per_rank, r["executions_by_rank"]
    assert len(r["llm_calls_by_rank"]) >= world // 2, r["llm_calls_by_rank"]


def test_load_balancer_moves_queued_task_across_ranks():
    r = run(4, "lb_move")
    assert r["moved"] == 2
    moved = [t for t in r["queued_ids"] if t in r["dst_queue"]]
    assert len(moved) == 2 and len(r["src_queue"]) == 1
    assert not set(moved) & set(r["src_queue"])
    # an agent-level stop leaves the worker rank serving (it used to end the rank's plane loop)
    assert r["lost_after_agent_stop"] == [] and r["rank1_alive"] and r["rank1_serving"]


def test_dynamic_scaling_creates_agent_on_least_loaded_rank():
    r = run(4, "scale")
    assert r["registered"] and r["scaled_ok"]
    assert r["new_rank"] in (1, 2, 3)  # rank 0 was made to look busy


def test_rank_loss_requeues_and_completes_every_task_exactly_once():
    """Rank 2 dies mid-run (os._exit in the middle of its third task): the plane detects
    it, its in-flight tasks are re-queued on the survivors, its agents leave the pool, and
    every submitted task completes exactly once."""
    r = run(4, "kill", per_rank=2)
    assert r["exitcodes"][2] == 17 and r["exitcodes"][0] == 0, r["exitcodes"]
    assert r["lost_ranks"] == [2]
    assert r["succeeded"] == r["submitted"] == 40
    assert r["completed_ids"] == r["unique_completed"] == 40
    assert r["requeued"] >= 1
    assert r["agents_after"] == 6


async def test_plane_refuses_unauthenticated_and_duplicate_hellos():
    """a hello must carry the job's shared secret and claim a rank that is in range
    and not already alive; a refused duplicate must not take down the live rank's state."""
    import asyncio

    from pilottai_amd.parallel.node_plane import PlaneServer, PlaneWorker, _recv, _send
    from pilottai_amd.parallel.node_rehearsal import free_port

    port = free_port()
    srv = PlaneServer(3, port=port, hb_timeout=30.0, secret="s3cret")
    srv._server = await asyncio.start_server(srv._handle, srv.host, srv.port)

    async def raw_hello(**hello):
        r, w = await asyncio.open_connection("127.0.0.1", port)
        await _send(w, {"op": "hello", **hello})
        try:
            await asyncio.wait_for(_recv(r), 1.0)
            return "open"
        except (asyncio.IncompleteReadError, ConnectionError):
            return "closed"
        except asyncio.TimeoutError:
            return "open"
        finally:
            w.close()

    assert await raw_hello(rank=1, secret="wrong") == "closed"
    assert await raw_hello(rank=7, secret="s3cret") == "closed"  # outside the world
    assert await raw_hello(rank=0, secret="s3cret") == "closed"  # rank 0 is the server
    good = PlaneWorker(1, [], port=port, secret="s3cret")
    await good.connect(timeout=5)
    for _ in range(50):
        if 1 in srv.ranks and srv.ranks[1].alive:
            break
        await asyncio.sleep(0.02)
    live = srv.ranks[1]
    assert live.alive
    assert await raw_hello(rank=1, secret="s3cret") == "closed"  # duplicate of a live rank
    await asyncio.sleep(0.1)
    assert srv.ranks[1] is live and live.alive and srv.lost == []
    assert srv.rejected == 4
    good._writer.close()
    srv._server.close()


def test_plane_capacity_at_world8_matches_independent_ranks():
    """64 closed-loop clients at world 8 with every LLM call taking the
    per-call latency of an 8-worker rank (80 ms). One manager on rank 0 over the node-wide
    pool (--dp-mode node) must keep up with 8 independent Serves: measured 0.96-1.0x on this
    container; rank 0's event loop stays responsive (10 ms sleep probe)."""
    node = run(8, "throughput", per_rank=8, latency=0.08)
    indep = run(8, "throughput_indep", per_rank=8, latency=0.08)
    assert node["exitcodes"] == [0] * 8 and indep["exitcodes"] == [0] * 8
    assert indep["tasks_per_s"] > 100, indep  # ~20 tasks/s per rank: 5 dependent 80 ms calls per task
    # (0.96-1.0x on an idle container; 0.94 when the test tier runs on parallel workers that
    # share the 8 CPUs with these 16 processes, hence the 0.9 floor)
    assert node["tasks_per_s"] >= 0.9 * indep["tasks_per_s"], (node["tasks_per_s"], indep["tasks_per_s"])
    assert node["loop_lag_ms_p99"] < 50, node
