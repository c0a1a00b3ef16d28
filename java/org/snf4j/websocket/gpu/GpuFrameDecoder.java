/*
 * The "ws-decoder" stage on the MI355X: FrameDecoder (FrameDecoder.java:41-403)
 * with FrameUtf8Validator (FrameUtf8Validator.java:59-98) fused, decoded in
 * cross-session device batches (WsgBatcher).
 *
 * available() is the reference's frame delimiting, on the loop thread
 * (FrameDecoder.java:290-401, through wsg_frame_available).  decode() hands the
 * bytes to the batcher and releases `data` exactly once (FrameDecoder.java:285-287);
 * it returns with `out` empty.  The frames come back in deliver(), on the
 * session's loop thread, and go through the decoders after "ws-decoder" and the
 * handler, in order.  The first error does what FrameDecoder.java:92-102 does:
 * writenf(CloseFrame(code)), the closed latch, and an InvalidFrameException with
 * the reference's message (GENTLE close, InvalidFrameException.java:75-77).
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;

import org.snf4j.core.codec.IBaseDecoder;
import org.snf4j.core.codec.ICodec;
import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.core.codec.IDecoder;
import org.snf4j.core.session.ISession;
import org.snf4j.core.session.IStreamSession;
import org.snf4j.websocket.IWebSocketSessionConfig;
import org.snf4j.websocket.frame.CloseFrame;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.InvalidFrameException;

public class GpuFrameDecoder implements IBaseDecoder<ByteBuffer, Frame> {

	private final WsgBatcher batcher;
	private final boolean clientMode, allowExtensions;
	private final int maxPayloadLen;
	final int sid;
	long nativeBatcher;
	private ISession session;
	/** FrameDecoder.closed (:63): after the first error all input is swallowed. */
	private boolean closed;
	/** bytes of the current frame still to come (FrameDecoder.availablePayload, :348-355) */
	private long remaining;
	private final long[] err = new long[4];

	public GpuFrameDecoder(boolean clientMode, boolean allowExtensions, int maxPayloadLen, boolean validateUtf8,
			WsgBatcher batcher) {
		this.batcher = batcher;
		this.clientMode = clientMode;
		this.allowExtensions = allowExtensions;
		this.maxPayloadLen = maxPayloadLen;
		this.sid = batcher.register(this, clientMode, allowExtensions, maxPayloadLen, validateUtf8);
	}

	@Override
	public Class<ByteBuffer> getInboundType() {
		return ByteBuffer.class;
	}

	@Override
	public Class<Frame> getOutboundType() {
		return Frame.class;
	}

	ISession session() {
		return session;
	}

	/** FrameDecoder.available(ISession, byte[], int, int) (FrameDecoder.java:357-401). */
	@Override
	public int available(ISession session, byte[] buffer, int off, int len) {
		if (closed)
			return len;
		if (remaining > 0)
			return (int) Math.min(len, remaining);
		long r = Wsg.frameAvailable(buffer, off, len, err);
		return checked(session, r);
	}

	/** FrameDecoder.available(ISession, ByteBuffer, boolean) (:290-332); the buffer is not modified. */
	@Override
	public int available(ISession session, ByteBuffer buffer, boolean flipped) {
		ByteBuffer b = flipped ? buffer.duplicate() : (ByteBuffer) buffer.duplicate().flip();
		int len = b.remaining();
		if (closed)
			return len;
		if (remaining > 0)
			return (int) Math.min(len, remaining);
		long r;
		if (b.hasArray())
			r = Wsg.frameAvailable(b.array(), b.arrayOffset() + b.position(), len, err);
		else if (b.isDirect())
			r = Wsg.frameAvailableDirect(b, b.position(), len, err);
		else {  // (read-only heap buffer) the header copy of :310-331
			byte[] hdr = new byte[Math.min(len, 14)];
			b.get(hdr);
			r = Wsg.frameAvailable(hdr, 0, len, err);
		}
		return checked(session, r);
	}

	/** err = {status, detail, detail2, frame length once the header is complete} */
	private int checked(ISession session, long r) {
		if (r < 0) {  // Negative / Extended payload length (FrameDecoder.java:388-394)
			fail(session, (int) err[0], err[1], err[2], true);
		}
		if (r > 0 && err[3] > r)  // a partial frame: the rest follows in later reads
			remaining = err[3];
		return (int) r;
	}

	/** FrameDecoder.decode (:180-288): the bytes go to the device batch. */
	@Override
	public void decode(ISession session, ByteBuffer data, List<Frame> out) throws Exception {
		try {
			this.session = session;
			if (closed)
				return;
			if (remaining > 0)
				remaining -= data.remaining();
			batcher.enqueue(this, session, data);
		} finally {
			session.release(data);
		}
	}

	/** The session's frames of one device batch, on its loop thread. */
	void deliver(List<Frame> frames, int error, long detail) {
		if (closed)
			return;
		for (Frame f : frames)
			downstream(f);
		if (error != Wsg.OK)
			fail(session, error, detail, 0, false);
	}

	/** The decoders after "ws-decoder", then the handler (DefaultCodecExecutor.java:557-584). */
	@SuppressWarnings({ "unchecked", "rawtypes" })
	private void downstream(Frame frame) {
		ICodecPipeline pipeline = session.getCodecPipeline();
		List<Object> in = new ArrayList<Object>(1);
		in.add(frame);
		boolean after = false;
		for (Object key : pipeline.decoderKeys()) {
			if (!after) {
				after = IWebSocketSessionConfig.WEBSOCKET_DECODER.equals(key);
				continue;
			}
			ICodec<?, ?> c = pipeline.get(key);
			List<Object> next = new ArrayList<Object>();
			for (Object o : in) {
				try {
					((IDecoder) c).decode(session, o, next);
				} catch (Exception e) {
					session.getHandler().exception(e);
					session.close();
					return;
				}
			}
			in = next;
		}
		for (Object o : in)
			session.getHandler().read(o);
	}

	private void fail(ISession session, int status, long detail, long detail2, boolean inAvailable) {
		closed = true;
		remaining = 0;
		((IStreamSession) session).writenf(new CloseFrame(Wsg.closeCode(status)));
		InvalidFrameException e = new InvalidFrameException(Wsg.message(status, detail, detail2));
		if (inAvailable)
			throw e;  // FrameDecoder.available throws here too (:388-394)
		// a deferred decode error: what the selector loop does with the pipeline's exception
		// (InternalSelectorLoop.java:589-601), then the GENTLE close (InternalSession.java:804-829)
		session.getHandler().exception(e);
		session.close();
	}
}
