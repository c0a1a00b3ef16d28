/*
 * Cross-session batching of the frame codec (the host side of the MI355X codec).
 *
 * One WsgBatcher serves the sessions of one selector loop, on that loop's thread.
 * GpuFrameDecoder.decode() hands each read to enqueue(), which only records it (the
 * decoder's ownership of the buffer passes here: it is released once its bytes are
 * copied); GpuFrameEncoder.encode() queues each frame (wsg_enc_batcher_add copies
 * its payload).  The first of either in a loop iteration schedules flush() with
 * SelectorLoop.executenf, which QUEUES the task (InternalSelectorLoop.java:
 * 1002-1011, 1038-1046) — ISession.executenf would run it inline on the loop thread
 * (InternalSession.java:720-733) — so the flush runs in the loop's task phase
 * (InternalSelectorLoop.java:641, 751-758), after every read of the iteration.
 *
 * A flush, per native batcher:
 *   1. feeds the iteration's reads with ONE wsg_batcher_feed_many call (the native
 *      side copies them into the open batch's pinned arena and frames them, several
 *      threads for large iterations), then releases the buffers;
 *   2. delivers every earlier flush whose device work has finished (wsg_batcher_await
 *      with no wait; only with BATCHER_MAX_INFLIGHT (4) already in flight does it wait
 *      for the oldest);
 *   3. queues this iteration's batch (wsg_batcher_flush_async: H2D, decode + UTF-8 and
 *      the stages after the decoder, D2H) and hands its ticket to the completion
 *      thread.
 * The completion thread waits for the ticket (wsg_batcher_await: a host function on
 * the download stream signals it) and re-enters the loop with
 * executenf(collectTask), which wakes select(): the loop never blocks on the device
 * for the batch it just queued, and a batch is delivered in a later iteration even
 * when no further reads arrive.  The encode side is the same over wsg_enc_batcher_*;
 * a CLOSE frame first writes out everything in flight and queued (flushEncodes).
 * Frames go back to each session in flush order, through the rest of its codec
 * pipeline, as DefaultCodecExecutor.decode (DefaultCodecExecutor.java:557-584) and
 * CodecExecutorAdapter.read (CodecExecutorAdapter.java:228-254) would have passed
 * them; encoded bytes are written with session.writenf, which no Frame encoder
 * accepts, so they go to the socket as they are (DefaultCodecExecutor.java:390-410).
 * snf4j_amd/loop.py restates this scheduling in Python over the same C ABI; the GPU
 * tests run it against the oracle (tests/test_gpu_loop.py) and drive these natives
 * through the JNI glue (tests/test_gpu_jni.py).
 *
 * Session slots are reused: a decoder or encoder registers when its session first
 * sends or receives data and unregisters at the session's end (IEventDrivenCodec
 * ENDING / removed), which drops its unfed reads and resets the native slot
 * (wsg_batcher_session_reset, wsg_enc_batcher_session_reset; results of batches in
 * flight for the old session come back empty).  One device per loop: WsgDevices
 * hands the loops of a process out over the node's GPUs.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;
import java.util.ArrayDeque;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.HashMap;
import java.util.List;
import java.util.Map;
import java.util.concurrent.LinkedBlockingQueue;
import java.util.concurrent.TimeUnit;

import org.snf4j.core.SelectorLoop;
import org.snf4j.core.session.ISession;
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

	/** One native decode batcher, the decoders holding its slots and the iteration's reads. */
	private final class Native {
		final long handle;
		final GpuFrameDecoder[] slots;
		int next;
		/* the reads of this loop iteration (wsg_batcher_feed_many at the flush) */
		int nReads;
		int[] sids = new int[64], offs = new int[64], lens = new int[64];
		ByteBuffer[] direct = new ByteBuffer[64];
		byte[][] heap = new byte[64][];
		ByteBuffer[] owned = new ByteBuffer[64];   // released once fed (FrameDecoder.java:285-287)
		ISession[] owners = new ISession[64];
		/** tickets of the flushes on the device, oldest first */
		final ArrayDeque<Long> inflight = new ArrayDeque<Long>();

		Native(Cfg c) {
			handle = Wsg.batcherOpen(ctx, c.clientMode, c.allowExtensions, c.maxPayloadLen, c.validate, maxSessions);
			if (handle == 0)
				throw new IllegalStateException("wsg_batcher_open: " + Wsg.lastError(ctx));
			if (c.hasStages() && Wsg.batcherSetStages(handle, c.inflate, c.noContext, c.validate, c.aggregate,
					c.maxAggregatedLength) != 0)
				throw new IllegalStateException("wsg_batcher_set_stages: " + Wsg.lastError(ctx));
			if (Wsg.batcherReserve(handle, maxWireLen, maxFrames) != 0)
				throw new IllegalStateException("wsg_batcher_reserve: " + Wsg.lastError(ctx));
			// the stage chain's buffers too: inflated output up to STAGE_RATIO x the wire (more
			// grows on demand), within the 2 GiB a flush's payload view may span
			if (c.hasStages() && Wsg.batcherReserveStages(handle, maxStageLen(), maxFrames) != 0)
				throw new IllegalStateException("wsg_batcher_reserve_stages: " + Wsg.lastError(ctx));
			slots = new GpuFrameDecoder[maxSessions];
		}

		void grow() {
			int n = sids.length * 2;
			sids = Arrays.copyOf(sids, n);
			offs = Arrays.copyOf(offs, n);
			lens = Arrays.copyOf(lens, n);
			direct = Arrays.copyOf(direct, n);
			heap = Arrays.copyOf(heap, n);
			owned = Arrays.copyOf(owned, n);
			owners = Arrays.copyOf(owners, n);
		}
	}

	/** One encode flush on the device: its ticket and the encoders with frames in it. */
	private static final class EncFlush {
		final long ticket;
		final List<GpuFrameEncoder> encoders;

		EncFlush(long ticket, List<GpuFrameEncoder> encoders) {
			this.ticket = ticket;
			this.encoders = encoders;
		}
	}

	/**
	 * One native encode batcher: wsg_enc_batcher_open takes the client mode, and a batcher
	 * with the permessage-deflate-encoder stage (wsg_enc_batcher_set_deflate) one
	 * PerMessageDeflateEncoder(level, noContext) configuration.
	 */
	private final class EncNative {
		final long handle;
		final GpuFrameEncoder[] slots;
		int next;
		/** the encoders with frames in the open batch (each once: GpuFrameEncoder.openBatch) */
		List<GpuFrameEncoder> open = new ArrayList<GpuFrameEncoder>();
		long serial = 1;  // the open batch's number
		final ArrayDeque<EncFlush> inflight = new ArrayDeque<EncFlush>();

		EncNative(boolean clientMode, GpuPerMessageDeflateEncoder deflate) {
			handle = Wsg.encBatcherOpen(ctx, clientMode, maxSessions);
			if (handle == 0)
				throw new IllegalStateException("wsg_enc_batcher_open: " + Wsg.lastError(ctx));
			if (deflate != null && Wsg.encBatcherSetDeflate(handle, deflate.level, deflate.noContext) != 0)
				throw new IllegalStateException("wsg_enc_batcher_set_deflate: " + Wsg.lastError(ctx));
			if (Wsg.encBatcherReserve(handle, maxFrames, maxWireLen) != 0)
				throw new IllegalStateException("wsg_enc_batcher_reserve: " + Wsg.lastError(ctx));
			slots = new GpuFrameEncoder[maxSessions];
		}
	}

	/**
	 * The completion thread: waits for the flushes it is given (wsg_batcher_await /
	 * wsg_enc_batcher_await, the only natives called off the loop thread) and re-enters
	 * the loop with executenf(collectTask) for each.
	 */
	private final class Completion extends Thread {
		private final LinkedBlockingQueue<long[]> watch = new LinkedBlockingQueue<long[]>();
		volatile boolean stopped;

		Completion() {
			super("wsg-completion-" + loop.getId());
			setDaemon(true);
		}

		void watch(long handle, long ticket, boolean encode) {
			watch.add(new long[] {handle, ticket, encode ? 1 : 0});
		}

		@Override
		public void run() {
			while (!stopped) {
				long[] w;
				try {
					w = watch.poll(100, TimeUnit.MILLISECONDS);
				} catch (InterruptedException e) {
					return;
				}
				if (w == null)
					continue;
				while (!stopped) {
					long done = w[2] != 0 ? Wsg.encBatcherAwait(w[0], w[1] - 1, 100) : Wsg.batcherAwait(w[0], w[1] - 1, 100);
					if (done < 0 || done >= w[1])  // (a native error: the loop's collect reports it)
						break;
				}
				if (stopped)
					return;
				try {
					loop.executenf(collectTask);
				} catch (RuntimeException e) {  // SelectorLoopStoppingException: the loop is ending
					return;
				}
			}
		}
	}

	final long ctx;
	final int device;
	private final boolean ownsDevice;
	private final SelectorLoop loop;
	private final int maxSessions;
	private final long maxFrames, maxWireLen;
	private final Map<Cfg, Native> natives = new HashMap<Cfg, Native>();
	/* by encNativeIndex: client mode, then no deflate stage or its level and noContext */
	private final EncNative[] encNatives = new EncNative[2 * 21];
	private boolean flushScheduled;
	private final Completion completion;
	private final ByteBuffer[] views = new ByteBuffer[5];
	private final long[] counts = new long[2];
	private final Runnable flushTask = new Runnable() {
		@Override
		public void run() {
			flush();
		}
	};
	private final Runnable collectTask = new Runnable() {
		@Override
		public void run() {
			collectReady();
		}
	};

	/**
	 * @param loop        the selector loop whose sessions this batcher serves
	 * @param device      HIP device index (WsgDevices.deviceFor(loop) spreads loops over the GPUs)
	 * @param maxSessions sessions of the selector loop
	 * @param maxFrames   frames a flush may hold (workspace and staging reserved once:
	 *                    wsg_reserve, wsg_batcher_reserve, wsg_enc_batcher_reserve)
	 * @param maxWireLen  wire bytes a flush may hold
	 */
	public WsgBatcher(SelectorLoop loop, int device, int maxSessions, long maxFrames, long maxWireLen) {
		this(loop, device, false, maxSessions, maxFrames, maxWireLen);
	}

	/** A batcher on the device WsgDevices assigns to the loop (given back by close()). */
	public WsgBatcher(SelectorLoop loop, int maxSessions, long maxFrames, long maxWireLen) {
		this(loop, WsgDevices.deviceFor(loop), true, maxSessions, maxFrames, maxWireLen);
	}

	private WsgBatcher(SelectorLoop loop, int device, boolean ownsDevice, int maxSessions, long maxFrames,
			long maxWireLen) {
		// a flush's payload region is handed to Java as one direct buffer (< 2 GiB)
		if (maxWireLen + 16 * maxFrames + 16 > Integer.MAX_VALUE)
			throw new IllegalArgumentException("maxWireLen + 16 * maxFrames must stay below 2 GiB");
		if (loop == null)
			throw new IllegalArgumentException("loop is null");
		ctx = Wsg.open(device);
		if (ctx == 0)
			throw new IllegalStateException("wsg_open(" + device + ") failed");
		this.device = device;
		this.ownsDevice = ownsDevice;
		this.loop = loop;
		this.maxSessions = maxSessions;
		this.maxFrames = maxFrames;
		this.maxWireLen = maxWireLen;
		if (Wsg.reserve(ctx, maxFrames, maxSessions, maxWireLen) != 0)
			throw new IllegalStateException("wsg_reserve: " + Wsg.lastError(ctx));
		completion = new Completion();
		completion.start();
	}

	/** Inflated bytes a flush's stages are sized for, per wire byte (permessage-deflate's typical ratio). */
	static final int STAGE_RATIO = 4;

	private long maxStageLen() {
		return Math.min(STAGE_RATIO * maxWireLen, Integer.MAX_VALUE - 16L * maxFrames - 32);
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

	private Native nativeOf(GpuFrameDecoder d) {
		for (Native n : natives.values())
			if (n.handle == d.nativeBatcher)
				return n;
		return null;
	}

	/** The session ended: its unfed reads are released, its slot free again with its carry dropped. */
	synchronized void unregister(GpuFrameDecoder d) {
		Native n = nativeOf(d);
		if (n == null || d.sid < 0 || n.slots[d.sid] != d)
			return;
		int k = 0;
		for (int i = 0; i < n.nReads; ++i) {
			if (n.sids[i] == d.sid) {
				n.owners[i].release(n.owned[i]);
				continue;
			}
			n.sids[k] = n.sids[i];
			n.offs[k] = n.offs[i];
			n.lens[k] = n.lens[i];
			n.direct[k] = n.direct[i];
			n.heap[k] = n.heap[i];
			n.owned[k] = n.owned[i];
			n.owners[k] = n.owners[i];
			++k;
		}
		for (int i = k; i < n.nReads; ++i) {
			n.direct[i] = null;
			n.heap[i] = null;
			n.owned[i] = null;
			n.owners[i] = null;
		}
		n.nReads = k;
		n.slots[d.sid] = null;
		Wsg.batcherSessionReset(n.handle, d.sid);
	}

	/**
	 * A session's read: recorded (the flush feeds it) and owned from here on — the
	 * buffer is released once its bytes are copied (FrameDecoder.java:285-287).
	 */
	synchronized void enqueue(GpuFrameDecoder d, ISession session, ByteBuffer data) {
		Native n = nativeOf(d);
		if (n == null) {
			session.release(data);
			return;
		}
		if (n.nReads == n.sids.length)
			n.grow();
		int i = n.nReads++;
		n.sids[i] = d.sid;
		if (data.isDirect()) {
			n.direct[i] = data;
			n.offs[i] = data.position();
		} else if (data.hasArray()) {
			n.heap[i] = data.array();
			n.offs[i] = data.arrayOffset() + data.position();
		} else {  // a read-only heap buffer: no array, no address
			byte[] b = new byte[data.remaining()];
			data.duplicate().get(b);
			n.heap[i] = b;
			n.offs[i] = 0;
		}
		n.lens[i] = data.remaining();
		n.owned[i] = data;
		n.owners[i] = session;
		schedule();
	}

	/**
	 * Every frame d's session has read so far delivered now, in order: the iteration's
	 * reads of d's batcher fed and flushed, and all its flushes collected, waiting for
	 * the device.  GpuFrameDecoder.available calls it before it throws a header error
	 * (FrameDecoder.java:388-394), since the reference delivered the frames before that
	 * header when it reached it.  An error path: the loop blocks here.
	 */
	synchronized void drain(GpuFrameDecoder d) {
		Native n = nativeOf(d);
		if (n == null)
			return;
		try {
			boolean fed = n.nReads > 0;
			feedReads(n);
			if (fed) {
				if (n.inflight.size() == Wsg.BATCHER_MAX_INFLIGHT)
					collectOldest(n);
				check(Wsg.batcherFlushAsync(n.handle), "wsg_batcher_flush_async");
				n.inflight.add(Wsg.batcherTicket(n.handle));
			}
			while (!n.inflight.isEmpty())
				collectOldest(n);
		} catch (RuntimeException ex) {
			failSessions(n, ex);
		}
	}

	/* ------------------------------------------------------------------ encode side */

	private static int encNativeIndex(boolean clientMode, GpuPerMessageDeflateEncoder deflate) {
		int d = deflate == null ? 0 : 1 + 2 * deflate.level + (deflate.noContext ? 1 : 0);
		return 2 * d + (clientMode ? 1 : 0);
	}

	/**
	 * A session slot for an encoder (at its first queued frame), in a fresh state; with
	 * deflate (the session's GPU permessage-deflate-encoder) a slot of the batcher running
	 * that configuration, with a new deflater.
	 */
	synchronized int registerEncoder(GpuFrameEncoder e, boolean clientMode, GpuPerMessageDeflateEncoder deflate) {
		int m = encNativeIndex(clientMode, deflate);
		if (encNatives[m] == null)
			encNatives[m] = new EncNative(clientMode, deflate);
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

	private EncNative encNativeOf(GpuFrameEncoder e) {
		for (EncNative n : encNatives)
			if (n != null && n.handle == e.nativeBatcher)
				return n;
		return null;
	}

	synchronized void unregisterEncoder(GpuFrameEncoder e) {
		EncNative n = encNativeOf(e);
		if (n != null && e.sid >= 0 && n.slots[e.sid] == e) {
			n.slots[e.sid] = null;
			Wsg.encBatcherSessionReset(n.handle, e.sid);  // its queued and in-flight frames are dropped
		}
	}

	/** Queue a frame of the encoder's session; it is written by a later flush. */
	synchronized void enqueueEncode(GpuFrameEncoder e, Frame frame, int mask) {
		EncNative n = encNativeOf(e);
		int flags = (frame.isFinalFragment() ? 0x80 : 0) | ((frame.getRsvBits() & 7) << 4);
		int rc = Wsg.encBatcherAdd(e.nativeBatcher, e.sid, frame.getOpcode().value(), flags, mask, frame.getPayload());
		if (rc != 0)
			throw new IllegalStateException("wsg_enc_batcher_add: " + rc);
		if (e.openBatch != n.serial) {  // first frame of e in the open batch
			e.openBatch = n.serial;
			e.batches++;
			n.open.add(e);
		}
		schedule();
	}

	/** True if the encoder's session has frames queued or on the device (later frames queue behind them). */
	boolean hasQueued(GpuFrameEncoder e) {
		return e.batches > 0;
	}

	/* ------------------------------------------------------------------ flush */

	private void schedule() {
		if (!flushScheduled) {
			flushScheduled = true;
			loop.executenf(flushTask);  // queued: runs after this iteration's reads
		}
	}

	/** The loop iteration's batches (see the class comment). */
	synchronized void flush() {
		flushScheduled = false;
		for (Native n : natives.values()) {
			boolean fed = n.nReads > 0;
			try {
				feedReads(n);
				collectReady(n);
				if (!fed)
					continue;
				if (n.inflight.size() == Wsg.BATCHER_MAX_INFLIGHT)
					collectOldest(n);
				check(Wsg.batcherFlushAsync(n.handle), "wsg_batcher_flush_async");
				long t = Wsg.batcherTicket(n.handle);
				n.inflight.add(t);
				completion.watch(n.handle, t, false);
			} catch (RuntimeException ex) {
				failSessions(n, ex);
			}
		}
		for (EncNative n : encNatives) {
			if (n == null)
				continue;
			try {
				collectReady(n);
				if (n.open.isEmpty())
					continue;
				if (n.inflight.size() == 2)
					writeOldest(n);
				check(Wsg.encBatcherFlushAsync(n.handle), "wsg_enc_batcher_flush_async");
				long t = Wsg.encBatcherTicket(n.handle);
				n.inflight.add(new EncFlush(t, n.open));
				n.open = new ArrayList<GpuFrameEncoder>();
				n.serial++;
				completion.watch(n.handle, t, true);
			} catch (RuntimeException ex) {
				failSessions(n, ex);
			}
		}
	}

	private static void check(int rc, String what) {
		if (rc != 0)
			throw new IllegalStateException(what + ": " + rc);
	}

	/** The iteration's reads in one native call, then their buffers released. */
	private void feedReads(Native n) {
		if (n.nReads == 0)
			return;
		int rc = Wsg.batcherFeedMany(n.handle, n.nReads, n.sids, n.direct, n.heap, n.offs, n.lens);
		for (int i = 0; i < n.nReads; ++i) {
			n.owners[i].release(n.owned[i]);
			n.direct[i] = null;
			n.heap[i] = null;
			n.owned[i] = null;
			n.owners[i] = null;
		}
		n.nReads = 0;
		check(rc, "wsg_batcher_feed_many");
	}

	/** collectTask (re-entered by the completion thread): every finished flush. */
	synchronized void collectReady() {
		for (Native n : natives.values()) {
			try {
				collectReady(n);
			} catch (RuntimeException ex) {
				failSessions(n, ex);
			}
		}
		for (EncNative n : encNatives) {
			if (n == null)
				continue;
			try {
				collectReady(n);
			} catch (RuntimeException ex) {
				failSessions(n, ex);
			}
		}
	}

	private void collectReady(Native n) {
		if (n.inflight.isEmpty())
			return;
		long done = Wsg.batcherAwait(n.handle, 0, 0);  // no wait: the highest finished ticket
		while (!n.inflight.isEmpty() && n.inflight.peek() <= done)
			collectOldest(n);
	}

	private void collectReady(EncNative n) {
		if (n.inflight.isEmpty())
			return;
		long done = Wsg.encBatcherAwait(n.handle, 0, 0);
		while (!n.inflight.isEmpty() && n.inflight.peek().ticket <= done)
			writeOldest(n);
	}

	/** The oldest decode flush of n (waits if it is not done): frames to their sessions. */
	private void collectOldest(Native n) {
		n.inflight.poll();
		check(Wsg.batcherWait(n.handle, views, counts), "wsg_batcher_wait");
		WsgDevices.account(device, counts[1]);
		ByteBuffer sf = views[0].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer desc = views[1].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer payload = views[2];
		ByteBuffer result = views[3].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer detail2 = views[4].order(ByteOrder.LITTLE_ENDIAN);
		for (int sid = 0; sid < maxSessions; ++sid) {
			GpuFrameDecoder d = n.slots[sid];
			if (d == null)
				continue;
			final int delivered = result.getInt(Wsg.RESULT_BYTES * sid);
			final int error = result.getShort(Wsg.RESULT_BYTES * sid + 4) & 0xffff;
			if (delivered == 0 && error == Wsg.OK)
				continue;
			final int first = sf.getInt(4 * sid);
			final long detail = result.getLong(Wsg.RESULT_BYTES * sid + 8);
			final long d2 = detail2.getLong(8 * sid);  // Extended payload length's bound (:393)
			final List<Frame> frames = new ArrayList<Frame>(delivered);
			for (int i = 0; i < delivered; ++i)
				frames.add(frame(desc, payload, first + i));
			// on the loop thread that owns the session (this batcher's loop); the views are
			// reused by a later flush, so frames own byte[] copies (Frame.java:53)
			d.deliver(frames, error, detail, d2);
		}
	}

	/**
	 * Encode every queued frame and write it now (an encoder calls this before it writes
	 * a CLOSE frame, so what was written before the CLOSE goes out first).
	 */
	synchronized void flushEncodes() {
		for (EncNative n : encNatives) {
			if (n == null)
				continue;
			while (!n.inflight.isEmpty())
				writeOldest(n);
			if (n.open.isEmpty())
				continue;
			check(Wsg.encBatcherFlush(n.handle, views), "wsg_enc_batcher_flush");
			List<GpuFrameEncoder> es = n.open;
			n.open = new ArrayList<GpuFrameEncoder>();
			n.serial++;
			write(n, es);
		}
	}

	/** The oldest in-flight encode flush of n (waits if it is not done): bytes to the sockets. */
	private void writeOldest(EncNative n) {
		EncFlush f = n.inflight.poll();
		check(Wsg.encBatcherWait(n.handle, views), "wsg_enc_batcher_wait");
		write(n, f.encoders);
	}

	/** Each encoder's frames of a flush's views, in one buffer, to its session. */
	private void write(EncNative n, List<GpuFrameEncoder> es) {
		ByteBuffer sf = views[0].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer off = views[1].order(ByteOrder.LITTLE_ENDIAN);
		ByteBuffer wire = views[2];
		for (GpuFrameEncoder e : es) {
			e.batches--;
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

	/**
	 * A native call failed (a device or allocation error, never a protocol error): the
	 * sessions of that batcher get the exception and close, as a failing codec pipeline
	 * closes its session (InternalSelectorLoop.java:589-601), instead of the loop logging
	 * it and the sessions waiting for frames that never come.
	 */
	private void failSessions(Native n, RuntimeException ex) {
		n.inflight.clear();
		for (GpuFrameDecoder d : n.slots)
			if (d != null)
				d.failBatch(ex);
	}

	private void failSessions(EncNative n, RuntimeException ex) {
		n.inflight.clear();
		for (GpuFrameEncoder e : n.slots)
			if (e != null)
				e.failBatch(ex);
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

	/**
	 * Stops the completion thread, delivers what is in flight, frees the native batchers
	 * and the device context, and gives the loop's device back when WsgDevices assigned it.
	 */
	public void close() {
		completion.stopped = true;
		completion.interrupt();
		try {
			completion.join();
		} catch (InterruptedException e) {
			Thread.currentThread().interrupt();
		}
		synchronized (this) {
			for (Native n : natives.values()) {
				for (int i = 0; i < n.nReads; ++i)  // reads never fed: their buffers released
					n.owners[i].release(n.owned[i]);
				n.nReads = 0;
				while (!n.inflight.isEmpty())
					collectOldest(n);
				Wsg.batcherClose(n.handle);
			}
			natives.clear();
			for (int i = 0; i < encNatives.length; ++i)
				if (encNatives[i] != null) {
					while (!encNatives[i].inflight.isEmpty())  // the device work ends before the batcher does
						writeOldest(encNatives[i]);
					Wsg.encBatcherClose(encNatives[i].handle);
					encNatives[i] = null;
				}
			Wsg.close(ctx);
			if (ownsDevice)
				WsgDevices.release(loop);
		}
	}
}
