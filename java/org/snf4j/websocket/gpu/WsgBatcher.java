/*
 * Cross-session batching of the frame codec (the host side of the MI355X codec).
 *
 * One WsgBatcher serves the sessions of one selector loop, on that loop's thread.
 * GpuFrameDecoder.decode() feeds each session's bytes (wsg_batcher_feed copies them
 * and does the host framing); GpuFrameEncoder.encode() queues each frame
 * (wsg_enc_batcher_add copies its payload).  The first of either in a loop
 * iteration schedules flush() with SelectorLoop.executenf, which QUEUES the task
 * (InternalSelectorLoop.java:1002-1011, 1038-1046) — ISession.executenf would run it
 * inline on the loop thread (InternalSession.java:720-733) — so the flush runs in the
 * loop's task phase (InternalSelectorLoop.java:641, 751-758), after every read of
 * the iteration: one device batch per native batcher for every session that read
 * (gather to pinned staging, H2D, decode + UTF-8 kernels and the batched stages
 * after them, D2H), then one encode batch for every session that wrote, queued on
 * the device and written to the sockets by the next iteration's flush (the loop does
 * not wait for it; a CLOSE frame first writes out everything before it).  Frames
 * go back to each session in order, through the rest of its codec pipeline, as
 * DefaultCodecExecutor.decode (DefaultCodecExecutor.java:557-584) and
 * CodecExecutorAdapter.read (CodecExecutorAdapter.java:228-254) would have passed
 * them; encoded bytes are written with session.writenf, which no Frame encoder
 * accepts, so they go to the socket as they are (DefaultCodecExecutor.java:390-410).
 *
 * Session slots are reused: a decoder or encoder registers when its session first
 * sends or receives data and unregisters at the session's end (IEventDrivenCodec
 * ENDING / removed), which resets the native slot (wsg_batcher_session_reset,
 * wsg_enc_batcher_session_reset).  One device per loop: WsgDevices hands the loops
 * of a process out over the node's GPUs.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.LinkedHashSet;
import java.util.List;
import java.util.Map;
import java.util.Set;

import org.snf4j.core.SelectorLoop;
import org.snf4j.core.session.IStreamSession;
import org.snf4j.websocket.frame.AggregatedBinaryFrame;
import org.snf4j.websocket.frame.AggregatedTextFrame;
import org.snf4j.websocket.frame.BinaryFrame;
import org.snf4j.websocket.frame.CloseFrame;
import org.snf4j.websocket.frame.ContinuationFrame;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.PingFrame;
import org.snf4j.websocket.frame.PongFrame;
import org.snf4j.websocket.frame.TextFrame;

public final class WsgBatcher {

	/**
	 * A decoder configuration: FrameDecoder constructor arguments, fused validation and
	 * the batched stages after the decoder (wsg_batcher_open and wsg_batcher_set_stages
	 * take one each).
	 */
	static final class Cfg {
		final boolean clientMode, allowExtensions, validate;
		final int maxPayloadLen;
		final boolean inflate, noContext, aggregate;
		final int maxAggregatedLength;

		Cfg(boolean clientMode, boolean allowExtensions, int maxPayloadLen, boolean validate, boolean inflate,
				boolean noContext, boolean aggregate, int maxAggregatedLength) {
			this.clientMode = clientMode;
			this.allowExtensions = allowExtensions;
			this.maxPayloadLen = maxPayloadLen;
			this.validate = validate;
			this.inflate = inflate;
			this.noContext = noContext;
			this.aggregate = aggregate;
			this.maxAggregatedLength = maxAggregatedLength;
		}

		boolean hasStages() {
			return inflate || aggregate;
		}

		@Override
		public boolean equals(Object o) {
			if (!(o instanceof Cfg))
				return false;
			Cfg c = (Cfg) o;
			return c.clientMode == clientMode && c.allowExtensions == allowExtensions && c.validate == validate
					&& c.maxPayloadLen == maxPayloadLen && c.inflate == inflate && c.noContext == noContext
					&& c.aggregate == aggregate && c.maxAggregatedLength == maxAggregatedLength;
		}

		@Override
		public int hashCode() {
			return (clientMode ? 1 : 0) | (allowExtensions ? 2 : 0) | (validate ? 4 : 0) | (inflate ? 8 : 0)
					| (noContext ? 16 : 0) | (aggregate ? 32 : 0) | (maxPayloadLen << 6) ^ maxAggregatedLength;
		}
	}

	/** One native decode batcher and the decoders holding its slots. */
	private final class Native {
		final long handle;
		final GpuFrameDecoder[] slots;
		int next;
		final Set<GpuFrameDecoder> dirty = new LinkedHashSet<GpuFrameDecoder>();

		Native(Cfg c) {
			handle = Wsg.batcherOpen(ctx, c.clientMode, c.allowExtensions, c.maxPayloadLen, c.validate, maxSessions);
			if (handle == 0)
				throw new IllegalStateException("wsg_batcher_open: " + Wsg.lastError(ctx));
			if (c.hasStages() && Wsg.batcherSetStages(handle, c.inflate, c.noContext, c.validate, c.aggregate,
					c.maxAggregatedLength) != 0)
				throw new IllegalStateException("wsg_batcher_set_stages: " + Wsg.lastError(ctx));
			slots = new GpuFrameDecoder[maxSessions];
		}
	}

	/** One native encode batcher (wsg_enc_batcher_open takes the client mode). */
	private final class EncNative {
		final long handle;
		final GpuFrameEncoder[] slots;
		int next;
		final Set<GpuFrameEncoder> dirty = new LinkedHashSet<GpuFrameEncoder>();
		/** The encoders of each flush on the device (wsg_enc_batcher_flush_async), oldest first. */
		final ArrayDeque<List<GpuFrameEncoder>> inflight = new ArrayDeque<List<GpuFrameEncoder>>();

		EncNative(boolean clientMode) {
			handle = Wsg.encBatcherOpen(ctx, clientMode, maxSessions);
			if (handle == 0)
				throw new IllegalStateException("wsg_enc_batcher_open: " + Wsg.lastError(ctx));
			slots = new GpuFrameEncoder[maxSessions];
		}
	}

	final long ctx;
	final int device;
	private final SelectorLoop loop;
	private final int maxSessions;
	private final Map<Cfg, Native> natives = new HashMap<Cfg, Native>();
	private final EncNative[] encNatives = new EncNative[2];
	private boolean flushScheduled;
	private final Runnable flushTask = new Runnable() {
		@Override
		public void run() {
			flush();
		}
	};

	/**
	 * @param loop        the selector loop whose sessions this batcher serves
	 * @param device      HIP device index (WsgDevices.deviceFor(loop) spreads loops over the GPUs)
	 * @param maxSessions sessions of the selector loop
	 * @param maxFrames   frames a flush may hold (workspace reserved once, wsg_reserve)
	 * @param maxWireLen  wire bytes a flush may hold
	 */
	public WsgBatcher(SelectorLoop loop, int device, int maxSessions, long maxFrames, long maxWireLen) {
		// a flush's payload region is handed to Java as one direct buffer (< 2 GiB)
		if (maxWireLen + 16 * maxFrames + 16 > Integer.MAX_VALUE)
			throw new IllegalArgumentException("maxWireLen + 16 * maxFrames must stay below 2 GiB");
		if (loop == null)
			throw new IllegalArgumentException("loop is null");
		ctx = Wsg.open(device);
		if (ctx == 0)
			throw new IllegalStateException("wsg_open(" + device + ") failed");
		this.device = device;
		this.loop = loop;
		this.maxSessions = maxSessions;
		if (Wsg.reserve(ctx, maxFrames, maxSessions, maxWireLen) != 0)
			throw new IllegalStateException("wsg_reserve: " + Wsg.lastError(ctx));
	}

	/** A batcher on the device WsgDevices assigns to the loop. */
	public WsgBatcher(SelectorLoop loop, int maxSessions, long maxFrames, long maxWireLen) {
		this(loop, WsgDevices.deviceFor(loop), maxSessions, maxFrames, maxWireLen);
	}

	/* ------------------------------------------------------------------ decode side */

	/** A session slot for a decoder (at its first decode), in a fresh state. */
	synchronized int register(GpuFrameDecoder d, Cfg c) {
		Native n = natives.get(c);
		if (n == null) {
			n = new Native(c);
			natives.put(c, n);
		}
		for (int i = 0; i < maxSessions; ++i) {
			int sid = (n.next + i) % maxSessions;
			if (n.slots[sid] == null) {
				if (Wsg.batcherSessionReset(n.handle, sid) != 0)
					throw new IllegalStateException("wsg_batcher_session_reset: " + sid);
				n.slots[sid] = d;
				n.next = sid + 1;
				d.nativeBatcher = n.handle;
				return sid;
			}
		}
		throw new IllegalStateException("no free session slot (maxSessions " + maxSessions + ")");
	}

	/** The session ended: its slot is free again, with its bytes and carry dropped. */
	synchronized void unregister(GpuFrameDecoder d) {
		for (Native n : natives.values())
			if (n.handle == d.nativeBatcher && d.sid >= 0 && n.slots[d.sid] == d) {
				n.slots[d.sid] = null;
				n.dirty.remove(d);
				Wsg.batcherSessionReset(n.handle, d.sid);
			}
	}

	/** Feed a session's bytes and make sure a flush runs after this loop iteration. */
	synchronized void enqueue(GpuFrameDecoder d, ByteBuffer data) {
		int rc;
		if (data.hasArray())
			rc = Wsg.batcherFeedArray(d.nativeBatcher, d.sid, data.array(), data.arrayOffset() + data.position(),
					data.remaining());
		else if (data.isDirect())
			rc = Wsg.batcherFeed(d.nativeBatcher, d.sid, data, data.position(), data.remaining());
		else {  // a read-only heap buffer: no array, no address
			byte[] b = new byte[data.remaining()];
			data.duplicate().get(b);
			rc = Wsg.batcherFeedArray(d.nativeBatcher, d.sid, b, 0, b.length);
		}
		if (rc != 0)
			throw new IllegalStateException("wsg_batcher_feed: " + rc);
		for (Native n : natives.values())
			if (n.handle == d.nativeBatcher)
				n.dirty.add(d);
		schedule();
	}

	/* ------------------------------------------------------------------ encode side */

	synchronized int registerEncoder(GpuFrameEncoder e, boolean clientMode) {
		int m = clientMode ? 1 : 0;
		if (encNatives[m] == null)
			encNatives[m] = new EncNative(clientMode);
		EncNative n = encNatives[m];
		for (int i = 0; i < maxSessions; ++i) {
			int sid = (n.next + i) % maxSessions;
			if (n.slots[sid] == null) {
				if (Wsg.encBatcherSessionReset(n.handle, sid) != 0)
					throw new IllegalStateException("wsg_enc_batcher_session_reset: " + sid);
				n.slots[sid] = e;
				n.next = sid + 1;
				e.nativeBatcher = n.handle;
				return sid;
			}
		}
		throw new IllegalStateException("no free encoder slot (maxSessions " + maxSessions + ")");
	}

	synchronized void unregisterEncoder(GpuFrameEncoder e) {
		for (EncNative n : encNatives)
			if (n != null && n.handle == e.nativeBatcher && e.sid >= 0 && n.slots[e.sid] == e) {
				n.slots[e.sid] = null;
				n.dirty.remove(e);
				Wsg.encBatcherSessionReset(n.handle, e.sid);
			}
	}

	/** Queue a frame of the encoder's session; it is written by the next flush. */
	synchronized void enqueueEncode(GpuFrameEncoder e, Frame frame, int mask) {
		int flags = (frame.isFinalFragment() ? 0x80 : 0) | ((frame.getRsvBits() & 7) << 4);
		int rc = Wsg.encBatcherAdd(e.nativeBatcher, e.sid, frame.getOpcode().value(), flags, mask, frame.getPayload());
		if (rc != 0)
			throw new IllegalStateException("wsg_enc_batcher_add: " + rc);
		for (EncNative n : encNatives)
			if (n != null && n.handle == e.nativeBatcher)
				n.dirty.add(e);
		schedule();
	}

	/** True if the encoder's session has frames queued or on the device (later frames must queue behind them). */
	synchronized boolean hasQueued(GpuFrameEncoder e) {
		for (EncNative n : encNatives) {
			if (n == null)
				continue;
			if (n.dirty.contains(e))
				return true;
			for (List<GpuFrameEncoder> f : n.inflight)
				if (f.contains(e))
					return true;
		}
		return false;
	}

	/* ------------------------------------------------------------------ flush */

	private void schedule() {
		if (!flushScheduled) {
			flushScheduled = true;
			loop.executenf(flushTask);  // queued: runs after this iteration's reads
		}
	}

	/**
	 * One device batch per native batcher; frames go back to their sessions, bytes to
	 * the sockets.  The decode batches are queued first (wsg_batcher_flush_async); the
	 * encode batch queued by the previous flush is written out and this iteration's is
	 * queued (wsg_enc_batcher_flush_async: its bytes go out one loop iteration later,
	 * so the loop does not wait for its H2D, kernels and D2H); then each decode is
	 * collected.
	 */
	synchronized void flush() {
		flushScheduled = false;
		List<Native> queued = new ArrayList<Native>();
		for (Native n : natives.values()) {
			if (n.dirty.isEmpty())
				continue;
			int rc = Wsg.batcherFlushAsync(n.handle);
			if (rc != 0)
				throw new IllegalStateException("wsg_batcher_flush_async: " + rc);
			queued.add(n);
		}
		flushEncodesAsync();
		collectDecodes(queued);
	}

	private void collectDecodes(List<Native> queued) {
		ByteBuffer[] views = new ByteBuffer[5];
		long[] counts = new long[2];
		for (Native n : queued) {
			int rc = Wsg.batcherWait(n.handle, views, counts);
			if (rc != 0)
				throw new IllegalStateException("wsg_batcher_wait: " + rc);
			WsgDevices.account(device, counts[1]);
			ByteBuffer sf = views[0].order(ByteOrder.LITTLE_ENDIAN);
			ByteBuffer desc = views[1].order(ByteOrder.LITTLE_ENDIAN);
			ByteBuffer payload = views[2];
			ByteBuffer result = views[3].order(ByteOrder.LITTLE_ENDIAN);
			ByteBuffer detail2 = views[4].order(ByteOrder.LITTLE_ENDIAN);
			List<GpuFrameDecoder> ds = new ArrayList<GpuFrameDecoder>(n.dirty);
			n.dirty.clear();
			for (GpuFrameDecoder d : ds) {
				final int first = sf.getInt(4 * d.sid);
				final int delivered = result.getInt(Wsg.RESULT_BYTES * d.sid);
				final int error = result.getShort(Wsg.RESULT_BYTES * d.sid + 4) & 0xffff;
				final long detail = result.getLong(Wsg.RESULT_BYTES * d.sid + 8);
				final long d2 = detail2.getLong(8 * d.sid);  // Extended payload length's bound (:393)
				final List<Frame> frames = new ArrayList<Frame>(delivered);
				for (int i = 0; i < delivered; ++i)
					frames.add(frame(desc, payload, first + i));
				// on the loop thread that owns the session (this batcher's loop); the views are
				// reused by the next flush, so frames own byte[] copies (Frame.java:53)
				d.deliver(frames, error, detail, d2);
			}
		}
	}

	/**
	 * Encode every queued frame and write it now (an encoder calls this before it writes
	 * a CLOSE frame, so what was written before the CLOSE goes out first).
	 */
	synchronized void flushEncodes() {
		ByteBuffer[] views = new ByteBuffer[3];
		for (EncNative n : encNatives) {
			if (n == null)
				continue;
			while (!n.inflight.isEmpty())
				collectEncode(n, views);
			if (n.dirty.isEmpty())
				continue;
			int rc = Wsg.encBatcherFlush(n.handle, views);
			if (rc != 0)
				throw new IllegalStateException("wsg_enc_batcher_flush: " + rc);
			List<GpuFrameEncoder> es = new ArrayList<GpuFrameEncoder>(n.dirty);
			n.dirty.clear();
			write(n, es, views);
		}
	}

	/** The flush's step for the encode side: the previous flush's bytes out, this one's queued. */
	private void flushEncodesAsync() {
		ByteBuffer[] views = new ByteBuffer[3];
		for (EncNative n : encNatives) {
			if (n == null)
				continue;
			while (!n.inflight.isEmpty())
				collectEncode(n, views);
			if (n.dirty.isEmpty())
				continue;
			int rc = Wsg.encBatcherFlushAsync(n.handle);
			if (rc != 0)
				throw new IllegalStateException("wsg_enc_batcher_flush_async: " + rc);
			n.inflight.add(new ArrayList<GpuFrameEncoder>(n.dirty));
			n.dirty.clear();
			schedule();  // the next iteration's flush writes it out, whatever else arrives
		}
	}

	/** The oldest in-flight encode flush of n: its bytes to their sessions' sockets. */
	private void collectEncode(EncNative n, ByteBuffer[] views) {
		int rc = Wsg.encBatcherWait(n.handle, views);
		if (rc != 0)
			throw new IllegalStateException("wsg_enc_batcher_wait: " + rc);
		write(n, n.inflight.poll(), views);
	}

	/** Each encoder's frames of a flush's views, in one buffer, to its session. */
	private void write(EncNative n, List<GpuFrameEncoder> es, ByteBuffer[] views) {
		ByteBuffer sf = views[0].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer off = views[1].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer wire = views[2];
		for (GpuFrameEncoder e : es) {
			// a session reset since (unregister, slot reuse) dropped its frames from the view
			if (e.sid < 0 || n.slots[e.sid] != e)
				continue;
			long from = off.getLong(8 * sf.getInt(4 * e.sid)), to = off.getLong(8 * sf.getInt(4 * (e.sid + 1)));
			int len = (int) (to - from);
			IStreamSession session = e.session();
			if (len == 0 || session == null)
				continue;
			ByteBuffer out = session.allocate(len);  // FrameEncoder.java:78: the session's allocator
			ByteBuffer src = wire.duplicate();
			src.position((int) from).limit((int) to);
			out.put(src).flip();
			session.writenf(out);  // no Frame encoder takes a ByteBuffer: straight to the socket
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
		if ((flags & Wsg.OUT_AGGREGATED) != 0)  // FrameAggregator's message (FrameAggregator.java:76-99)
			return opcode == 1 ? new AggregatedTextFrame(true, rsv, data) : new AggregatedBinaryFrame(true, rsv, data);
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
		for (int i = 0; i < encNatives.length; ++i)
			if (encNatives[i] != null) {
				while (!encNatives[i].inflight.isEmpty()) {  // the device work ends before the batcher does
					Wsg.encBatcherWait(encNatives[i].handle, null);
					encNatives[i].inflight.poll();
				}
				Wsg.encBatcherClose(encNatives[i].handle);
				encNatives[i] = null;
			}
		Wsg.close(ctx);
	}
}
