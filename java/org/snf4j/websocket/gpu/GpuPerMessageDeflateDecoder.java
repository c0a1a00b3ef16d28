/*
 * The permessage-deflate decoder (PerMessageDeflateDecoder.java:33-107 over
 * DeflateDecoder.java:78-141) on the MI355X.  In the decoder's device batch
 * (wsg_inflate_batch_*, inflate.hip: k_infl_tok / k_infl_fast / k_inflate) when it
 * directly follows the GPU decoder, which is where PerMessageDeflateExtension puts
 * it ("permessage-deflate-decoder" after "ws-decoder",
 * PerMessageDeflateExtension.java:316-326); the inflater state and 32 KiB window
 * then live in the native batcher, per session.  Otherwise the wrapped reference
 * decoder runs, with its own zlib inflater and session-event handling.
 */
package org.snf4j.websocket.gpu;

import java.util.List;

import org.snf4j.core.codec.ICodecPipeline;
import org.snf4j.core.codec.IDecoder;
import org.snf4j.core.codec.IEventDrivenCodec;
import org.snf4j.core.handler.SessionEvent;
import org.snf4j.core.session.ISession;
import org.snf4j.websocket.extensions.compress.PerMessageDeflateDecoder;
import org.snf4j.websocket.frame.Frame;

public class GpuPerMessageDeflateDecoder implements IDecoder<Frame, Frame>, IEventDrivenCodec, GpuStage {

	final boolean noContext;
	private final PerMessageDeflateDecoder fallback;
	private boolean batched;

	public GpuPerMessageDeflateDecoder(boolean noContext, PerMessageDeflateDecoder fallback) {
		this.noContext = noContext;
		this.fallback = fallback != null ? fallback : new PerMessageDeflateDecoder(noContext);
	}

	@Override
	public Class<Frame> getInboundType() {
		return Frame.class;
	}

	@Override
	public Class<Frame> getOutboundType() {
		return Frame.class;
	}

	@Override
	public void setBatched() {
		batched = true;
	}

	@Override
	public boolean isBatched() {
		return batched;
	}

	@Override
	public void decode(ISession session, Frame frame, List<Frame> out) throws Exception {
		if (batched)
			out.add(frame);  // (inflated in the device batch)
		else
			fallback.decode(session, frame, out);
	}

	@Override
	public void added(ISession session, ICodecPipeline pipeline) {
		fallback.added(session, pipeline);
	}

	@Override
	public void event(ISession session, SessionEvent event) {
		fallback.event(session, event);  // (the batched state is dropped by GpuFrameDecoder's slot reset)
	}

	@Override
	public void removed(ISession session, ICodecPipeline pipeline) {
		fallback.removed(session, pipeline);
	}
}
