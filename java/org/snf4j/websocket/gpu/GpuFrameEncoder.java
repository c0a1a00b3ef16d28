/*
 * The "ws-encoder" stage: FrameEncoder (FrameEncoder.java:41-136) with the header
 * emit and the client-side masking done on the MI355X for every session of the
 * selector loop in one device batch per loop iteration (WsgBatcher,
 * wsg_enc_batcher_*: k_enc_* kernels).
 *
 * encode() runs on the loop thread (EncodeTask.java:216-245).  A frame from the
 * device threshold up (4 KiB by default, so configs' 64 KiB fragments all go to
 * the device) is queued and encode() returns with `out` empty; the batch is
 * written to the session after the loop iteration's reads (session.writenf of the
 * encoded bytes, which no Frame encoder takes).  Smaller frames are header bytes
 * plus a short copy: they go through the reference FrameEncoder on the spot,
 * unless frames of the session are already queued, in which case they queue
 * behind them so the session's frames keep their order.  A CLOSE frame first
 * writes everything queued (the closing handshake, WebSocketSession.CloseTask,
 * writes it right before session.close()), then latches (:71-76).  Masks come
 * from a java.util.Random as FrameEncoder.RANDOM draws them (:43,111).
 *
 * With a GPU permessage-deflate-encoder in front (GpuPerMessageDeflateExtension puts a
 * GpuPerMessageDeflateEncoder under "permessage-deflate-encoder" and attaches it here),
 * compression is a stage of the same device batch (wsg_enc_batcher_set_deflate): the
 * marker hands frames on unchanged and every data frame (TEXT / BINARY / CONTINUATION,
 * whatever its size: each one moves the session's deflater or its compressing flag,
 * PerMessageDeflateEncoder.java:83-99) is queued; control frames, which the deflate
 * encoder passes through, keep the threshold rule above.
 *
 * Write futures: for a queued frame encode() returns with `out` empty, and snf4j's
 * EncodeTask completes the write's future at once (EncodeTask.java:380-381), before
 * the bytes are encoded or written.  So session.write(frame).sync() on a frame at or
 * above the device threshold only says the frame was queued; an application that
 * needs a write confirmation per frame sets the threshold above its largest frame
 * (the reference FrameEncoder then encodes on the spot) or waits for a later frame's
 * future below the threshold, which is written after the queued ones.  A device
 * failure reaches the session as an exception and closes it (failBatch); frames
 * queued or in flight when the session ends are dropped, as its unwritten bytes are.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.util.List;
import java.util.Random;

import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.core.codec.IEncoder;
import org.snf4j.core.codec.IEventDrivenCodec;
import org.snf4j.core.handler.SessionEvent;
import org.snf4j.core.session.ISession;
import org.snf4j.core.session.IStreamSession;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.FrameEncoder;
import org.snf4j.websocket.frame.Opcode;

public class GpuFrameEncoder implements IEncoder<Frame, ByteBuffer>, IEventDrivenCodec {

	private static final Random RANDOM = new Random();
	public static final int DEFAULT_DEVICE_THRESHOLD = 4096;
	/** frames with at least this many payload bytes are encoded on the device */
	private final int deviceThreshold;
	private final boolean clientMode;
	private final FrameEncoder small;
	private final WsgBatcher batcher;
	int sid = -1;
	long nativeBatcher;
	/** WsgBatcher bookkeeping: the open batch this encoder last added to, and the batches
	 * (open or on the device) holding its frames */
	long openBatch;
	int batches;
	private IStreamSession session;
	/** FrameEncoder.closed (:71-76) */
	private boolean closed;
	/** the batched permessage-deflate-encoder in front of this encoder, or null */
	private GpuPerMessageDeflateEncoder deflate;
	private boolean released;

	public GpuFrameEncoder(boolean clientMode, WsgBatcher batcher, int deviceThreshold) {
		this.clientMode = clientMode;
		this.batcher = batcher;
		this.deviceThreshold = deviceThreshold;
		this.small = new FrameEncoder(clientMode);
	}

	public GpuFrameEncoder(boolean clientMode, WsgBatcher batcher) {
		this(clientMode, batcher, DEFAULT_DEVICE_THRESHOLD);
	}

	@Override
	public Class<Frame> getInboundType() {
		return Frame.class;
	}

	@Override
	public Class<ByteBuffer> getOutboundType() {
		return ByteBuffer.class;
	}

	IStreamSession session() {
		return session;
	}

	/**
	 * The session's permessage-deflate-encoder runs in this encoder's device batch (called
	 * when the extension installs it, before any frame of the session is encoded).
	 */
	void attachDeflate(GpuPerMessageDeflateEncoder d) {
		if (sid >= 0 || deflate != null)
			return;  // frames already went out without it: the marker keeps its reference encoder
		deflate = d;
		d.setBatched();
	}

	@Override
	public void encode(ISession session, Frame frame, List<ByteBuffer> out) throws Exception {
		this.session = (IStreamSession) session;
		if (closed || released)
			return;  // FrameEncoder.java:71-76
		if (frame.getOpcode() == Opcode.CLOSE) {
			if (sid >= 0 && batcher.hasQueued(this))
				batcher.flushEncodes();  // what was written before the CLOSE goes out first
			small.encode(session, frame, out);
			closed = true;
			return;
		}
		boolean queued = sid >= 0 && batcher.hasQueued(this);
		boolean data = !frame.getOpcode().isControl();
		if (frame.getPayloadLength() < deviceThreshold && !queued && !(deflate != null && data)) {
			small.encode(session, frame, out);
			return;
		}
		if (sid < 0)
			sid = batcher.registerEncoder(this, clientMode, deflate);
		batcher.enqueueEncode(this, frame, clientMode ? RANDOM.nextInt() : 0);
	}

	/** The device batch holding this session's frames failed: the session gets the exception and closes. */
	void failBatch(Exception e) {
		if (released || session == null)
			return;
		closed = true;
		session.getHandler().exception(e);
		session.close();
	}

	/* ---- IEventDrivenCodec: the slot goes back at the session's end ---- */

	@Override
	public void added(ISession session, ICodecPipeline pipeline) {
		this.session = (IStreamSession) session;
	}

	@Override
	public void event(ISession session, SessionEvent event) {
		if (event == SessionEvent.ENDING)
			release();
	}

	@Override
	public void removed(ISession session, ICodecPipeline pipeline) {
		release();
	}

	private void release() {
		if (!released) {
			released = true;
			if (sid >= 0)
				batcher.unregisterEncoder(this);
		}
	}
}
