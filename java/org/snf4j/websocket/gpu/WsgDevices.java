/*
 * Which GPU serves which selector loop.
 *
 * The reference decodes each session on its own loop (one decoder per session,
 * DefaultWebSocketSessionConfig.java:276-281; a session belongs to one loop), so
 * sessions shard across GPUs by loop with nothing shared between devices: each
 * WsgBatcher opens one device and batches the sessions of one loop (DESIGN.md §6,
 * no collective).  The policy is native and process-wide (wsg_device_for_loop,
 * batcher.hip): a new loop goes to the device with the fewest loops, ties to the
 * one that has decoded the fewest wire bytes (the byte balance ShardPlan uses for a
 * node-wide batch, snf4j_amd/shard.py); a loop keeps its device until released,
 * since its sessions' carry state lives in that device's batcher.
 */
package org.snf4j.websocket.gpu;

import org.snf4j.core.SelectorLoop;

public final class WsgDevices {

	private WsgDevices() {
	}

	/** The device of `loop` (assigned on first use). */
	public static int deviceFor(SelectorLoop loop) {
		int d = Wsg.deviceForLoop(loop.getId());
		if (d < 0)
			throw new IllegalStateException("wsg_device_for_loop: no HIP device (" + d + ")");
		return d;
	}

	/** A batcher of `device` decoded `n` more wire bytes (the tie-break of deviceFor). */
	static void account(int device, long n) {
		Wsg.deviceAccount(device, n);
	}

	/** The loop stopped: its device serves one loop less. */
	public static void release(SelectorLoop loop) {
		Wsg.deviceReleaseLoop(loop.getId());
	}
}
