/*
 * Cross-session batching of the frame decoder (the host side of the MI355X codec).
 *
 * One WsgBatcher serves the sessions of one selector loop.  GpuFrameDecoder.decode()
 * feeds each session's bytes (wsg_batcher_feed copies them and does the host
 * framing); the first feed of a loop iteration schedules flush() with
 * ISession.executenf (ISession.java:368), so it runs on the loop thread after the
 * iteration's reads: one device batch (wsg_batcher_flush: gather to pinned
 * staging, H2D, decode + UTF-8 kernels, D2H) for every session that read.  The
 * frames then go back to each session on its own loop thread (executenf again)
 * and through the rest of its codec pipeline, as DefaultCodecExecutor.decode
 * (DefaultCodecExecutor.java:557-584) and CodecExecutorAdapter.read
 * (CodecExecutorAdapter.java:228-254) would have passed them.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import org.snf4j.core.session.ISession;
import org.snf4j.websocket.frame.BinaryFrame;
import org.snf4j.websocket.frame.CloseFrame;
import org.snf4j.websocket.frame.ContinuationFrame;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.PingFrame;
import org.snf4j.websocket.frame.PongFrame;
import org.snf4j.websocket.frame.TextFrame;

public final class WsgBatcher {

	/** A decoder configuration (FrameDecoder constructor arguments + fused validation). */
	private static final class Cfg {
		final boolean clientMode, allowExtensions, validate;
		final int maxPayloadLen;

		Cfg(boolean clientMode, boolean allowExtensions, int maxPayloadLen, boolean validate) {
			this.clientMode = clientMode;
			this.allowExtensions = allowExtensions;
			this.maxPayloadLen = maxPayloadLen;
			this.validate = validate;
		}

		@Override
		public boolean equals(Object o) {
			if (!(o instanceof Cfg))
				return false;
			Cfg c = (Cfg) o;
			return c.clientMode == clientMode && c.allowExtensions == allowExtensions && c.validate == validate
					&& c.maxPayloadLen == maxPayloadLen;
		}

		@Override
		public int hashCode() {
			return (clientMode ? 1 : 0) | (allowExtensions ? 2 : 0) | (validate ? 4 : 0) | (maxPayloadLen << 3);
		}
	}

	/** One native batcher (wsg_batcher_open takes one configuration) and its sessions. */
	private final class Native {
		final long handle;
		final GpuFrameDecoder[] slots;
		int used;
		final List<GpuFrameDecoder> dirty = new ArrayList<GpuFrameDecoder>();

		Native(Cfg c) {
			handle = Wsg.batcherOpen(ctx, c.clientMode, c.allowExtensions, c.maxPayloadLen, c.validate, maxSessions);
			if (handle == 0)
				throw new IllegalStateException("wsg_batcher_open: " + Wsg.lastError(ctx));
			slots = new GpuFrameDecoder[maxSessions];
		}
	}

	final long ctx;
	private final int maxSessions;
	private final Map<Cfg, Native> natives = new HashMap<Cfg, Native>();
	private boolean flushScheduled;
	private final Runnable flushTask = new Runnable() {
		@Override
		public void run() {
			flush();
		}
	};

	/**
	 * @param device      HIP device index
	 * @param maxSessions sessions of the selector loop
	 * @param maxFrames   frames a flush may hold (workspace reserved once, wsg_reserve)
	 * @param maxWireLen  wire bytes a flush may hold
	 */
	public WsgBatcher(int device, int maxSessions, long maxFrames, long maxWireLen) {
		// a flush's payload region is handed to Java as one direct buffer (< 2 GiB)
		if (maxWireLen + 16 * maxFrames + 16 > Integer.MAX_VALUE)
			throw new IllegalArgumentException("maxWireLen + 16 * maxFrames must stay below 2 GiB");
		ctx = Wsg.open(device);
		if (ctx == 0)
			throw new IllegalStateException("wsg_open(" + device + ") failed");
		this.maxSessions = maxSessions;
		if (Wsg.reserve(ctx, maxFrames, maxSessions, maxWireLen) != 0)
			throw new IllegalStateException("wsg_reserve: " + Wsg.lastError(ctx));
	}

	/** A session slot for a new decoder (called from GpuFrameDecoder's constructor). */
	synchronized int register(GpuFrameDecoder d, boolean clientMode, boolean allowExtensions, int maxPayloadLen,
			boolean validate) {
		Cfg c = new Cfg(clientMode, allowExtensions, maxPayloadLen, validate);
		Native n = natives.get(c);
		if (n == null) {
			n = new Native(c);
			natives.put(c, n);
		}
		for (int i = 0; i < maxSessions; ++i) {
			int sid = (n.used + i) % maxSessions;
			if (n.slots[sid] == null) {
				n.slots[sid] = d;
				n.used = sid + 1;
				d.nativeBatcher = n.handle;
				return sid;
			}
		}
		throw new IllegalStateException("no free session slot (maxSessions " + maxSessions + ")");
	}

	/** The session ended: its slot is free again (its carry state is reset on reuse by the caller). */
	synchronized void unregister(GpuFrameDecoder d) {
		for (Native n : natives.values())
			if (n.handle == d.nativeBatcher && n.slots[d.sid] == d)
				n.slots[d.sid] = null;
	}

	/** Feed a session's bytes and make sure a flush runs after this loop iteration. */
	synchronized void enqueue(GpuFrameDecoder d, ISession session, ByteBuffer data) {
		int rc;
		if (data.hasArray())
			rc = Wsg.batcherFeedArray(d.nativeBatcher, d.sid, data.array(), data.arrayOffset() + data.position(),
					data.remaining());
		else
			rc = Wsg.batcherFeed(d.nativeBatcher, d.sid, data, data.position(), data.remaining());
		if (rc != 0)
			throw new IllegalStateException("wsg_batcher_feed: " + rc);
		for (Native n : natives.values())
			if (n.handle == d.nativeBatcher && !n.dirty.contains(d))
				n.dirty.add(d);
		if (!flushScheduled) {
			flushScheduled = true;
			session.executenf(flushTask);
		}
	}

	/** One device batch per native batcher; frames go back to their sessions. */
	synchronized void flush() {
		flushScheduled = false;
		ByteBuffer[] views = new ByteBuffer[4];
		long[] counts = new long[2];
		for (Native n : natives.values()) {
			if (n.dirty.isEmpty())
				continue;
			int rc = Wsg.batcherFlush(n.handle, views, counts);
			if (rc != 0)
				throw new IllegalStateException("wsg_batcher_flush: " + rc);
			ByteBuffer sf = views[0].order(ByteOrder.LITTLE_ENDIAN);
			ByteBuffer desc = views[1].order(ByteOrder.LITTLE_ENDIAN);
			ByteBuffer payload = views[2];
			ByteBuffer result = views[3].order(ByteOrder.LITTLE_ENDIAN);
			for (GpuFrameDecoder d : n.dirty) {
				final int first = sf.getInt(4 * d.sid);
				final int delivered = result.getInt(Wsg.RESULT_BYTES * d.sid);
				final int error = result.getShort(Wsg.RESULT_BYTES * d.sid + 4) & 0xffff;
				final long detail = result.getLong(Wsg.RESULT_BYTES * d.sid + 8);
				final List<Frame> frames = new ArrayList<Frame>(delivered);
				for (int i = 0; i < delivered; ++i)
					frames.add(frame(desc, payload, first + i));
				final GpuFrameDecoder dec = d;
				// the views are reused by the next flush: frames own byte[] copies (Frame.java:53)
				d.session().executenf(new Runnable() {
					@Override
					public void run() {
						dec.deliver(frames, error, detail);
					}
				});
			}
			n.dirty.clear();
		}
	}

	/** Frame k of a flush, as FrameDecoder.createFrame builds it (FrameDecoder.java:104-157). */
	static Frame frame(ByteBuffer desc, ByteBuffer payload, int k) {
		final int base = Wsg.DESC_BYTES * k;
		final long off = desc.getLong(base);
		final int len = desc.getInt(base + 8);
		final int opcode = desc.get(base + 12) & 0x0f;
		final int flags = desc.get(base + 13) & 0xff;
		final boolean fin = (flags & 0x80) != 0;
		final int rsv = (flags >> 4) & 7;
		final byte[] data = new byte[len];
		ByteBuffer p = payload.duplicate();
		p.position((int) off);
		p.get(data);
		switch (opcode) {
		case 0: return new ContinuationFrame(fin, rsv, data);
		case 1: return new TextFrame(fin, rsv, data);
		case 2: return new BinaryFrame(fin, rsv, data);
		case 8: return new CloseFrame(rsv, data);
		case 9: return new PingFrame(rsv, data);
		default: return new PongFrame(rsv, data);
		}
	}

	/** Frees the device context and the native batchers. */
	public synchronized void close() {
		for (Native n : natives.values())
			Wsg.batcherClose(n.handle);
		natives.clear();
		Wsg.close(ctx);
	}
}
