/*
 * The "ws-decoder" stage on the MI355X: FrameDecoder (FrameDecoder.java:41-403)
 * decoded in cross-session device batches (WsgBatcher), with the GPU stages that
 * directly follow it in the pipeline run in the same batch: the UTF-8 check
 * (FrameUtf8Validator.java:59-98, fused into the decode kernels), or, when
 * permessage-deflate was negotiated, inflate then the validator
 * (PerMessageDeflateExtension.java:316-326), and an aggregator behind them.
 *
 * available() is the reference's frame delimiting, on the loop thread
 * (FrameDecoder.java:290-401, through wsg_frame_available).  decode() hands the
 * bytes, and the ownership of `data`, to the batcher, which releases it exactly once
 * after the loop iteration's flush has copied it (FrameDecoder.java:285-287); decode
 * returns with `out` empty.  The frames come back in deliver(), on the loop
 * thread, and go through the decoders after the batched stages and the handler, in
 * order.  The first error does what FrameDecoder.java:92-102 does:
 * writenf(CloseFrame(code)), the closed latch, and an InvalidFrameException with
 * the reference's message (GENTLE close, InvalidFrameException.java:75-77).
 *
 * An exception thrown after the decoder (a decoder behind the batched stages, or
 * the handler's read) ends the session as the selector loop ends it when the
 * pipeline throws (InternalSelectorLoop.java:589-601 -> InternalSession.exception
 * -> controlClose, InternalSession.java:804-848): an ICloseControllingException
 * GENTLE -> handler.exception(getClosingCause()) + close(); NONE -> the exception
 * only, the session goes on with its next frame; DEFAULT, or any other exception ->
 * handler.exception + quickClose().  Not reachable from outside org.snf4j.core:
 * futuresController.exception (the session futures fail when the session closes
 * instead) and pipelineItem.cause.
 *
 * available() throws the u64 length errors itself, as FrameDecoder.available does
 * (:388-394), but only after every frame the session read before the bad header
 * has been delivered (WsgBatcher.drain): the reference delivered those before it
 * reached the header.
 *
 * The session slot is taken at the first decode (the pipeline is then complete:
 * the handshake has switched the decoders and the extensions have added theirs)
 * and given back at the session's end (IEventDrivenCodec, as ZlibDecoder does,
 * ZlibDecoder.java:281-301), which resets it for the next session.
 */
package org.snf4j.websocket.gpu;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;

import org.snf4j.core.ICloseControllingException;
import org.snf4j.core.codec.IBaseDecoder;
import org.snf4j.core.codec.ICodec;
import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.core.codec.IDecoder;
import org.snf4j.core.codec.IEventDrivenCodec;
import org.snf4j.core.handler.IHandler;
import org.snf4j.core.handler.SessionEvent;
import org.snf4j.core.session.ISession;
import org.snf4j.core.session.IStreamSession;
import org.snf4j.websocket.IWebSocketSessionConfig;
import org.snf4j.websocket.frame.CloseFrame;
import org.snf4j.websocket.frame.Frame;
import org.snf4j.websocket.frame.InvalidFrameException;

public class GpuFrameDecoder implements IBaseDecoder<ByteBuffer, Frame>, IEventDrivenCodec {

	private final WsgBatcher batcher;
	private final boolean clientMode, allowExtensions;
	private final int maxPayloadLen;
	int sid = -1;
	long nativeBatcher;
	private ISession session;
	/** FrameDecoder.closed (:63): after the first error all input is swallowed. */
	private boolean closed;
	/** the session ended: the slot went back to the batcher */
	private boolean released;
	/** bytes of the current frame still to come (FrameDecoder.availablePayload, :348-355) */
	private long remaining;
	private final long[] err = new long[4];

	public GpuFrameDecoder(boolean clientMode, boolean allowExtensions, int maxPayloadLen, WsgBatcher batcher) {
		this.batcher = batcher;
		this.clientMode = clientMode;
		this.allowExtensions = allowExtensions;
		this.maxPayloadLen = maxPayloadLen;
	}

	@Override
	public Class<ByteBuffer> getInboundType() {
		return ByteBuffer.class;
	}

	@Override
	public Class<Frame> getOutboundType() {
		return Frame.class;
	}

	/** FrameDecoder.available(ISession, byte[], int, int) (FrameDecoder.java:357-401). */
	@Override
	public int available(ISession session, byte[] buffer, int off, int len) {
		if (closed)
			return len;
		if (remaining > 0)
			return (int) Math.min(len, remaining);
		long r = Wsg.frameAvailable(buffer, off, len, err);
		return checked(session, r, len);
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
			b.duplicate().get(hdr);  // available() must not move the buffer (IBaseDecoder.java:58-70)
			r = Wsg.frameAvailable(hdr, 0, len, err);
		}
		return checked(session, r, len);
	}

	/** err = {status, detail, detail2, frame length once the header is complete} */
	private int checked(ISession session, long r, int len) {
		if (r == -2)  // (the JNI call's arguments, never the bytes)
			throw new IllegalArgumentException("frameAvailable: bad buffer range");
		if (r < 0) {  // Negative / Extended payload length (FrameDecoder.java:388-394)
			long status = err[0], detail = err[1], detail2 = err[2];
			this.session = session;
			if (sid >= 0)
				batcher.drain(this);  // the frames read before this header first
			if (closed)  // one of them failed first: the reference never reached this header
				return len;
			fail(session, (int) status, detail, detail2, true);
		}
		if (r > 0 && err[3] > r)  // a partial frame: the rest follows in later reads
			remaining = err[3];
		return (int) r;
	}

	/**
	 * FrameDecoder.decode (:180-288): the bytes go to the device batch.  `data` is
	 * released exactly once (:285-287): here when it is swallowed, else by the batcher
	 * once the loop iteration's flush has copied it (WsgBatcher.enqueue).
	 */
	@Override
	public void decode(ISession session, ByteBuffer data, List<Frame> out) throws Exception {
		this.session = session;
		if (closed || released) {
			session.release(data);
			return;
		}
		try {
			if (sid < 0)
				sid = batcher.register(this, stages(session.getCodecPipeline()));
		} catch (RuntimeException e) {
			session.release(data);
			throw e;
		}
		if (remaining > 0)
			remaining -= data.remaining();
		batcher.enqueue(this, session, data);
	}

	/**
	 * The batch configuration: this decoder's arguments and the GPU stages that
	 * directly follow it, in the order the reference pipeline has them
	 * (permessage-deflate decoder, ws-utf8-validator, an aggregator); those are
	 * marked batched.
	 */
	private WsgBatcher.Cfg stages(ICodecPipeline pipeline) {
		List<ICodec<?, ?>> after = new ArrayList<ICodec<?, ?>>();
		boolean seen = false;
		for (Object key : pipeline.decoderKeys()) {
			if (seen)
				after.add(pipeline.get(key));
			else
				seen = IWebSocketSessionConfig.WEBSOCKET_DECODER.equals(key);
		}
		int i = 0;
		GpuPerMessageDeflateDecoder inflate = null;
		GpuFrameUtf8Validator validator = null;
		GpuFrameAggregator aggregator = null;
		if (i < after.size() && after.get(i) instanceof GpuPerMessageDeflateDecoder)
			inflate = (GpuPerMessageDeflateDecoder) after.get(i++);
		if (i < after.size() && after.get(i) instanceof GpuFrameUtf8Validator)
			validator = (GpuFrameUtf8Validator) after.get(i++);
		// the aggregator batches only behind the validator, or directly behind the decoder
		if ((validator != null || i == 0) && i < after.size() && after.get(i) instanceof GpuFrameAggregator)
			aggregator = (GpuFrameAggregator) after.get(i++);
		for (int k = 0; k < i; ++k)
			((GpuStage) after.get(k)).setBatched();
		return new WsgBatcher.Cfg(clientMode, allowExtensions, maxPayloadLen, validator != null, inflate != null,
				inflate != null && inflate.noContext, aggregator != null,
				aggregator != null ? aggregator.maxAggregatedLength : 0);
	}

	/** The session's frames of one device batch, on its loop thread. */
	void deliver(List<Frame> frames, int error, long detail, long detail2) {
		if (closed || released)
			return;
		List<IDecoder<Object, Object>> chain = chain();
		for (Frame f : frames)
			if (!downstream(f, chain))
				return;
		if (error != Wsg.OK)
			fail(session, error, detail, detail2, false);
	}

	/** The decoders after "ws-decoder" the batch did not run (once per delivery). */
	@SuppressWarnings("unchecked")
	private List<IDecoder<Object, Object>> chain() {
		ICodecPipeline pipeline = session.getCodecPipeline();
		List<IDecoder<Object, Object>> chain = new ArrayList<IDecoder<Object, Object>>();
		boolean after = false;
		for (Object key : pipeline.decoderKeys()) {
			if (!after) {
				after = IWebSocketSessionConfig.WEBSOCKET_DECODER.equals(key);
				continue;
			}
			ICodec<?, ?> c = pipeline.get(key);
			if (c instanceof GpuStage && ((GpuStage) c).isBatched())
				continue;
			chain.add((IDecoder<Object, Object>) c);
		}
		return chain;
	}

	/**
	 * One frame through the rest of the pipeline, then the handler
	 * (DefaultCodecExecutor.java:557-584, CodecExecutorAdapter.java:228-254).  An
	 * exception from either goes where the selector loop sends it (controlClose);
	 * false if the session is closed by it.
	 */
	private boolean downstream(Frame frame, List<IDecoder<Object, Object>> chain) {
		List<Object> in = new ArrayList<Object>(1);
		in.add(frame);
		try {
			for (IDecoder<Object, Object> c : chain) {
				List<Object> next = new ArrayList<Object>();
				for (Object o : in)
					c.decode(session, o, next);
				in = next;
			}
			for (Object o : in)
				session.getHandler().read(o);
		} catch (Exception e) {
			return controlClose(e);
		}
		return true;
	}

	/**
	 * InternalSession.exception / controlClose (InternalSession.java:804-848) for an
	 * exception the pipeline threw: true if the session stays open (close type NONE).
	 */
	private boolean controlClose(Throwable t) {
		IHandler handler = session.getHandler();
		if (t instanceof ICloseControllingException) {
			ICloseControllingException c = (ICloseControllingException) t;
			Throwable cause = c.getClosingCause();
			switch (c.getCloseType()) {
			case GENTLE:
				closed = true;
				handler.exception(cause);
				session.close();
				return false;
			case NONE:
				handler.exception(cause);
				return true;
			default:
				t = cause;
			}
		}
		closed = true;
		handler.exception(t);
		session.quickClose();
		return false;
	}

	/** The device batch this session's bytes were in failed (not a protocol error). */
	void failBatch(Exception e) {
		if (closed || released || session == null)
			return;
		controlClose(e);
	}

	private void fail(ISession session, int status, long detail, long detail2, boolean inAvailable) {
		closed = true;
		remaining = 0;
		((IStreamSession) session).writenf(new CloseFrame(Wsg.closeCode(status)));
		InvalidFrameException e = new InvalidFrameException(Wsg.message(status, detail, detail2));
		if (inAvailable)
			throw e;  // FrameDecoder.available throws here too (:388-394)
		// a deferred decode error: what the selector loop does with the pipeline's exception
		// (InternalSelectorLoop.java:589-601): InvalidFrameException is GENTLE (:75-77)
		controlClose(e);
	}

	/* ---- IEventDrivenCodec (IEventDrivenCodec.java:36-62) ---- */

	@Override
	public void added(ISession session, ICodecPipeline pipeline) {
		this.session = session;
	}

	/** The session is ending: its slot goes back to the batcher, reset for the next session. */
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
				batcher.unregister(this);
		}
	}
}
